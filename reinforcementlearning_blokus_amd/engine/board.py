"""Host-side Board (reference: engine/board.py).

The Board stays a Python object exactly like the reference's (numpy grid, Python-int
bitboards, per-player frontier ``set`` objects) because callers mutate it in place
and the reference's legal-move ORDER depends on the iteration order of those sets.
Every frontier mutation happens in the reference's sequence (update_frontier_after_move,
engine/board.py:315-367), so CPython lays the sets out identically and
``list(board.get_frontier(p))`` reproduces the reference order.

GPU work never reads this object directly: ``pack_state`` flattens it into the
256-byte ``bk_state`` record of include/blokus_hip.h, and ``frontier_tables`` carries
the same frontier sets as the library's restatement of CPython's hash tables (bk_fset,
kept in step with every place_piece / copy) for GPU playouts in the reference's
frontier order (``pack_fsets``).
"""
from __future__ import annotations

import logging
import os
from collections import defaultdict
from dataclasses import dataclass
from enum import Enum
from typing import Dict, List, Optional, Set, Tuple

import numpy as np

from .bitboard import coord_to_bit, coords_to_mask

logger = logging.getLogger(__name__)


class Player(Enum):
    RED = 1
    BLUE = 2
    YELLOW = 3
    GREEN = 4


_PLAYERS = list(Player)
_DIAG = ((-1, -1), (-1, 1), (1, -1), (1, 1))
_ORTH = ((-1, 0), (1, 0), (0, -1), (0, 1))


@dataclass
class Position:
    row: int
    col: int

    def __hash__(self):
        return hash((self.row, self.col))

    def __eq__(self, other):
        return self.row == other.row and self.col == other.col


class Board:
    """20x20 board: grid values 0 (empty) or Player.value."""

    SIZE = 20

    def __init__(self):
        n = self.SIZE
        self.grid = np.zeros((n, n), dtype=int)
        self.player_start_corners = {Player.RED: Position(0, 0), Player.BLUE: Position(0, n - 1),
                                     Player.YELLOW: Position(n - 1, n - 1), Player.GREEN: Position(n - 1, 0)}
        self.player_pieces_used = {p: set() for p in Player}
        self.player_first_move = dict.fromkeys(Player, True)
        self.game_over = False
        self.current_player = Player.RED
        self.move_count = 0
        self.player_frontiers: Dict[Player, Set[Tuple[int, int]]] = {p: set() for p in Player}
        self.init_frontiers()
        self.occupied_bits: int = 0
        self.player_bits: Dict[Player, int] = defaultdict(int)

    # ---------------------------------------------------------------- cells
    def is_valid_position(self, pos: Position) -> bool:
        return 0 <= pos.row < self.SIZE and 0 <= pos.col < self.SIZE

    def get_cell(self, pos: Position) -> int:
        return int(self.grid[pos.row, pos.col]) if self.is_valid_position(pos) else -1

    def set_cell(self, pos: Position, value: int) -> None:
        if self.is_valid_position(pos):
            self.grid[pos.row, pos.col] = value

    def is_empty(self, pos: Position) -> bool:
        return self.get_cell(pos) == 0

    def get_player_at(self, pos: Position) -> Optional[Player]:
        v = self.get_cell(pos)
        return None if v == 0 else Player(v)

    def _around(self, pos: Position, deltas) -> List[Position]:
        out = []
        for dr, dc in deltas:
            q = Position(pos.row + dr, pos.col + dc)
            if self.is_valid_position(q):
                out.append(q)
        return out

    def get_adjacent_positions(self, pos: Position) -> List[Position]:
        return self._around(pos, [(dr, dc) for dr in (-1, 0, 1) for dc in (-1, 0, 1) if dr or dc])

    def get_edge_adjacent_positions(self, pos: Position) -> List[Position]:
        return self._around(pos, _ORTH)

    def get_corner_adjacent_positions(self, pos: Position) -> List[Position]:
        return self._around(pos, _DIAG)

    def _has_neighbour(self, r: int, c: int, value: int, deltas) -> bool:
        g, n = self.grid, self.SIZE
        for dr, dc in deltas:
            rr, cc = r + dr, c + dc
            if 0 <= rr < n and 0 <= cc < n and g[rr, cc] == value:
                return True
        return False

    # ---------------------------------------------------------------- rules
    def can_place_piece(self, piece_positions: List[Position], player: Player) -> bool:
        """Grid legality (engine/board.py:136-173): on board, empty, covers the start
        corner on the first move, no edge contact with own cells, corner contact with
        own cells unless first move."""
        if not piece_positions:
            return False
        n, g = self.SIZE, self.grid
        for p in piece_positions:
            if not (0 <= p.row < n and 0 <= p.col < n) or g[p.row, p.col] != 0:
                return False
        if self.player_first_move[player] and self.player_start_corners[player] not in piece_positions:
            return False
        return self._check_adjacency_rules_fast(piece_positions, player.value, g)

    def _check_adjacency_rules(self, piece_positions: List[Position], player: Player) -> bool:
        return self._check_adjacency_rules_fast(piece_positions, player.value, self.grid)

    def _check_adjacency_rules_fast(self, piece_positions: List[Position], player_value: int, grid) -> bool:
        corner = False
        for p in piece_positions:
            if self._has_neighbour(p.row, p.col, player_value, _ORTH):
                return False
            corner = corner or self._has_neighbour(p.row, p.col, player_value, _DIAG)
        return corner or self.player_first_move[Player(player_value)]

    def _is_connected_via_corners(self, piece_positions: List[Position], player: Player) -> bool:
        if self.player_first_move[player]:
            return True
        return any(self._has_neighbour(p.row, p.col, player.value, _DIAG) for p in piece_positions)

    # ---------------------------------------------------------------- frontier
    def get_frontier(self, player: Player) -> Set[Tuple[int, int]]:
        """Live frontier set (do not mutate).  Its iteration order is the reference's."""
        return self.player_frontiers[player]

    def _compute_full_frontier(self, player: Player) -> Set[Tuple[int, int]]:
        v = player.value
        return {(r, c) for r in range(self.SIZE) for c in range(self.SIZE)
                if self.grid[r, c] == 0 and self._has_neighbour(r, c, v, _DIAG)
                and not self._has_neighbour(r, c, v, _ORTH)}

    def update_frontier_after_move(self, player: Player, placed_cells: List[Tuple[int, int]]) -> None:
        """Incremental update for the mover only; same add/discard sequence as the
        reference so the set layout (and list order) matches."""
        v, n, fr = player.value, self.SIZE, self.player_frontiers[player]
        for r, c in placed_cells:
            fr.discard((r, c))
            for dr, dc in _DIAG:
                rr, cc = r + dr, c + dc
                if 0 <= rr < n and 0 <= cc < n and self.grid[rr, cc] == 0 \
                        and not self._has_neighbour(rr, cc, v, _ORTH):
                    fr.add((rr, cc))
            for dr, dc in _ORTH:
                rr, cc = r + dr, c + dc
                if 0 <= rr < n and 0 <= cc < n:
                    fr.discard((rr, cc))

    def init_frontiers(self) -> None:
        for p in Player:
            self.player_frontiers[p].clear()
        for p in Player:
            self.init_frontier_for_player(p)
        from .._native import fset_new
        self.frontier_tables = fset_new(1)

    def init_frontier_for_player(self, player: Player) -> None:
        corner = self.player_start_corners[player]
        if self.is_empty(corner):
            self.player_frontiers[player].add((corner.row, corner.col))

    def debug_rebuild_frontier(self, player: Player) -> bool:
        full = self._compute_full_frontier(player)
        if full != self.player_frontiers[player]:
            logger.error("Frontier mismatch for %s", player.name)
            if os.getenv("BLOKUS_FRONTIER_DEBUG", ""):
                raise AssertionError(f"Frontier mismatch for {player.name}")
            self.player_frontiers[player] = full
            return False
        return True

    def _verify_frontier_consistency(self, player: Player) -> bool:
        v, corner = player.value, self.player_start_corners[player]
        for r, c in self.player_frontiers[player]:
            if self.grid[r, c] != 0:
                return False
            if self.player_first_move[player] and (r, c) == (corner.row, corner.col):
                continue
            if not self._has_neighbour(r, c, v, _DIAG) or self._has_neighbour(r, c, v, _ORTH):
                return False
        return True

    # ---------------------------------------------------------------- moves
    def place_piece(self, piece_positions: List[Position], player: Player, piece_id: int,
                    validate: bool = True) -> bool:
        if validate and not self.can_place_piece(piece_positions, player):
            return False
        cells = [(p.row, p.col) for p in piece_positions]
        for r, c in cells:
            self.grid[r, c] = player.value
        m = coords_to_mask(cells)
        self.occupied_bits |= m
        self.player_bits[player] |= m
        self.player_pieces_used[player].add(piece_id)
        self.player_first_move[player] = False
        self.update_frontier_after_move(player, cells)
        from .._native import fset_place
        fset_place(self.frontier_tables, _planes_record(self), player.value - 1, [r * 20 + c for r, c in cells])
        self.move_count += 1
        self._update_current_player()
        return True

    def _update_current_player(self) -> None:
        self.current_player = _PLAYERS[(_PLAYERS.index(self.current_player) + 1) % 4]

    # ---------------------------------------------------------------- scoring
    def get_score(self, player: Player) -> int:
        """Covered squares + 15 if all 21 pieces were used (engine/board.py:562-577)."""
        s = int(np.count_nonzero(self.grid == player.value))
        return s + 15 if len(self.player_pieces_used[player]) == 21 else s

    def get_winner(self) -> Optional[Player]:
        if not self.game_over:
            return None
        scores = {p: self.get_score(p) for p in Player}
        return max(scores, key=scores.get)

    def is_game_over(self) -> bool:
        return self.game_over

    def assert_bitboard_consistent(self) -> None:
        for r in range(self.SIZE):
            for c in range(self.SIZE):
                v = int(self.grid[r, c])
                bit = coord_to_bit(r, c)
                if bool(self.occupied_bits & bit) != (v != 0):
                    raise AssertionError(f"Bitboard inconsistency at ({r}, {c})")
                for p in Player:
                    if bool(self.player_bits[p] & bit) != (v == p.value):
                        raise AssertionError(f"Bitboard inconsistency at ({r}, {c}) for {p.name}")

    def copy(self) -> "Board":
        b = object.__new__(Board)
        b.grid = self.grid.copy()
        b.player_pieces_used = {k: v.copy() for k, v in self.player_pieces_used.items()}
        b.player_first_move = self.player_first_move.copy()
        b.game_over = self.game_over
        b.current_player = self.current_player
        b.move_count = self.move_count
        b.player_start_corners = self.player_start_corners
        b.player_frontiers = {k: v.copy() for k, v in self.player_frontiers.items()}
        from .._native import FSET_DTYPE, fset_copy
        b.frontier_tables = np.zeros(1, dtype=FSET_DTYPE)
        fset_copy(b.frontier_tables, self.frontier_tables)  # set.copy() re-lays out
        b.occupied_bits = self.occupied_bits
        b.player_bits = self.player_bits.copy()
        return b

    def __str__(self) -> str:
        return "\n".join("".join("." if v == 0 else str(int(v)) for v in row) for row in self.grid)


# --------------------------------------------------------------------- packing
def pack_state(board: Board, out=None):
    """Flatten a Board into one bk_state record (numpy STATE_DTYPE)."""
    from .._native import STATE_DTYPE
    rec = np.zeros(1, dtype=STATE_DTYPE) if out is None else out
    planes = np.zeros((4, 7), dtype=np.uint64)
    for i, p in enumerate(_PLAYERS):
        planes[i] = np.frombuffer(int(board.player_bits[p]).to_bytes(56, "little"), dtype="<u8")
    rec["planes"] = planes
    rec["used"] = [sum(1 << (pid - 1) for pid in board.player_pieces_used[p]) for p in _PLAYERS]
    rec["first_move"] = sum(int(board.player_first_move[p]) << i for i, p in enumerate(_PLAYERS))
    rec["current_player"] = board.current_player.value - 1
    rec["out_mask"] = 0
    rec["move_count"] = board.move_count
    return rec


def _planes_record(board: Board) -> np.ndarray:
    """bk_state with only the planes filled (what bk_fset_place reads)."""
    from .._native import STATE_DTYPE
    rec = np.zeros(1, dtype=STATE_DTYPE)
    for i, p in enumerate(_PLAYERS):
        rec["planes"][0, i] = np.frombuffer(int(board.player_bits[p]).to_bytes(56, "little"), dtype="<u8")
    return rec


def pack_fsets(boards) -> np.ndarray:
    """The boards' frontier tables (FSET_DTYPE), for bk_rollout_frontier."""
    from .._native import FSET_DTYPE
    out = np.zeros(len(boards), dtype=FSET_DTYPE)
    for i, b in enumerate(boards):
        out[i] = b.frontier_tables[0]
    return out


def pack_states(boards) -> np.ndarray:
    from .._native import STATE_DTYPE
    out = np.zeros(len(boards), dtype=STATE_DTYPE)
    for i, b in enumerate(boards):
        pack_state(b, out[i:i + 1])
    return out
