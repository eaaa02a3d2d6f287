"""Host-side 400-bit board masks (reference: engine/bitboard.py).

Cell (r, c) is bit r*20 + c of a Python int, exactly the reference layout
(engine/bitboard.py:19-22), so Board.player_bits / occupied_bits interoperate with
reference code.  The GPU kernels use a different, row-per-word layout internally;
only the packed bk_state (include/blokus_hip.h) crosses the boundary.
"""
from __future__ import annotations

from typing import Iterable, List, Optional, Tuple

BOARD_WIDTH = 20
BOARD_HEIGHT = 20
NUM_CELLS = BOARD_WIDTH * BOARD_HEIGHT

BIT_TABLE = [[1 << (BOARD_WIDTH * r + c) for c in range(BOARD_WIDTH)] for r in range(BOARD_HEIGHT)]
VALID_BOARD_MASK = (1 << NUM_CELLS) - 1

_ROW = (1 << BOARD_WIDTH) - 1
# column-band masks: _LEFT_COL_MASKS[n] = columns 0..n-1, _RIGHT_COL_MASKS[n] = the last n
_LEFT_COL_MASKS = [sum((((1 << n) - 1) << (BOARD_WIDTH * r)) for r in range(BOARD_HEIGHT))
                   for n in range(BOARD_WIDTH + 1)]
_RIGHT_COL_MASKS = [sum(((((1 << n) - 1) << (BOARD_WIDTH - n)) << (BOARD_WIDTH * r)) for r in range(BOARD_HEIGHT))
                    for n in range(BOARD_WIDTH + 1)]


def coord_to_index(row: int, col: int) -> int:
    return row * BOARD_WIDTH + col


def index_to_coord(index: int) -> Tuple[int, int]:
    return divmod(index, BOARD_WIDTH)


def coord_to_bit(row: int, col: int) -> int:
    return BIT_TABLE[row][col]


def coords_to_mask(coords: Iterable[Tuple[int, int]]) -> int:
    m = 0
    for r, c in coords:
        m |= BIT_TABLE[r][c]
    return m


def mask_to_coords(mask: int) -> List[Tuple[int, int]]:
    out = []
    while mask:
        low = mask & -mask
        out.append(index_to_coord(low.bit_length() - 1))
        mask ^= low
    return out


def shift_mask(mask: int, d_row: int, d_col: int, strict: bool = True) -> Optional[int]:
    """Move every set cell by (d_row, d_col).  strict: None if any cell leaves the
    board; otherwise such cells are dropped (engine/bitboard.py:125-170)."""
    out = 0
    for r, c in mask_to_coords(mask):
        nr, nc = r + d_row, c + d_col
        if 0 <= nr < BOARD_HEIGHT and 0 <= nc < BOARD_WIDTH:
            out |= BIT_TABLE[nr][nc]
        elif strict:
            return None
    return out


def shift_mask_fast(mask: int, d_row: int, d_col: int) -> int:
    """Non-strict shift with whole-int arithmetic (engine/bitboard.py:173-205): cells
    that would wrap a row edge are cleared first, then the int is shifted and clipped."""
    if not mask:
        return 0
    if d_col > 0:
        mask &= ~_RIGHT_COL_MASKS[min(d_col, BOARD_WIDTH)]
    elif d_col < 0:
        mask &= ~_LEFT_COL_MASKS[min(-d_col, BOARD_WIDTH)]
    s = d_row * BOARD_WIDTH + d_col
    mask = mask << s if s >= 0 else mask >> -s
    return mask & VALID_BOARD_MASK
