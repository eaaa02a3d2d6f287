"""LegalMoveGenerator on the MI355X (reference: engine/move_generator.py).

get_legal_moves computes the legal SET on the GPU (bk_movegen: dense 91x20 anchor
masks) and orders it on the host exactly as the reference does:

* frontier order (default, BLOKUS_USE_FRONTIER_MOVEGEN unset/1; _get_legal_moves_frontier,
  move_generator.py:261-559): piece asc, orientation asc, then the first (frontier cell,
  anchor index) that produced the move -- i.e. key min over the move's cells k lying on
  a frontier cell f of (rank of f in ``list(board.get_frontier(player))``, k);
* naive order (BLOKUS_USE_FRONTIER_MOVEGEN=0; _get_legal_moves_naive :153-259): piece,
  orientation, anchor row-major -- the order the dense masks already have.

There is no CPU move generator behind this class: without the HIP library or a GPU
every generation call raises NativeUnavailable.  Only single-move validation
(is_move_legal, used by BlokusGame.make_move) runs on the host.
"""
from __future__ import annotations

import logging
import os
import threading
from typing import List, Optional, Sequence

import numpy as np

from .bitboard import BIT_TABLE, coords_to_mask, mask_to_coords, shift_mask
from .board import Board, Player, Position
from .pieces import (ALL_PIECE_ORIENTATIONS, GID, ORIENT_CELLS, ORIENT_LIST, PieceGenerator,
                     PieceOrientation, PiecePlacement)

logger = logging.getLogger(__name__)


def _env_flag(name: str, default: bool) -> bool:
    raw = os.getenv(name)
    return default if raw is None else raw.lower() in ("1", "true", "yes", "on")


MOVEGEN_DEBUG = _env_flag("BLOKUS_MOVEGEN_DEBUG", False)
USE_FRONTIER_MOVEGEN = _env_flag("BLOKUS_USE_FRONTIER_MOVEGEN", True)
USE_BITBOARD_LEGALITY = _env_flag("BLOKUS_USE_BITBOARD_LEGALITY", True)   # accepted, no effect
USE_HEURISTIC_ANCHORS = _env_flag("BLOKUS_USE_HEURISTIC_ANCHORS", False)  # accepted, no effect
MOVEGEN_DEBUG_EQUIVALENCE = _env_flag("BLOKUS_MOVEGEN_DEBUG_EQUIVALENCE", False)
DEBUG_BITBOARD = _env_flag("BLOKUS_DEBUG_BITBOARD", False)

_PLAYERS = list(Player)

# per-orientation cell offsets as padded arrays (for vectorised ordering)
_NCELLS = np.array([len(c) for c in ORIENT_CELLS], dtype=np.int64)
_DR = np.zeros((len(ORIENT_CELLS), 5), dtype=np.int64)
_DC = np.zeros((len(ORIENT_CELLS), 5), dtype=np.int64)
for _g, _cells in enumerate(ORIENT_CELLS):
    for _k, (_r, _c) in enumerate(_cells):
        _DR[_g, _k], _DC[_g, _k] = _r, _c
_PID = np.array([p for p, _ in ORIENT_LIST], dtype=np.int64)
_OID = np.array([o for _, o in ORIENT_LIST], dtype=np.int64)
_BIG = 1 << 40


class Move:
    """A placement: piece id, orientation index, anchor (top-left of the bounding box)."""

    def __init__(self, piece_id: int, orientation: int, anchor_row: int, anchor_col: int):
        self.piece_id = piece_id
        self.orientation = orientation
        self.anchor_row = anchor_row
        self.anchor_col = anchor_col

    def get_positions(self, piece_orientations: List) -> List[Position]:
        shape = piece_orientations[self.orientation]
        return [Position(r, c) for r, c in PiecePlacement.get_piece_positions(shape, self.anchor_row, self.anchor_col)]

    def __str__(self):
        return (f"Move(piece_id={self.piece_id}, orientation={self.orientation}, "
                f"anchor=({self.anchor_row}, {self.anchor_col}))")

    __repr__ = __str__


def _rows_to_naive(rows: np.ndarray):
    """uint32[91,20] masks -> (g, r, c) arrays in naive order."""
    bits = np.unpackbits(np.ascontiguousarray(rows, dtype="<u4").view(np.uint8).reshape(91, 20, 4),
                         axis=2, bitorder="little")
    g, r, c = np.nonzero(bits)
    return g, r, c


def order_moves(rows: np.ndarray, frontier: Optional[Sequence] = None):
    """Order the legal moves of one board-player.

    rows: uint32[91,20] GPU masks.  frontier: iteration-order list of (row, col) of
    the player's frontier set, or None for naive order.  Returns (g, r, c) arrays.
    """
    g, r, c = _rows_to_naive(rows)
    if frontier is None or len(g) == 0:
        return g, r, c
    rank = np.full(400, _BIG, dtype=np.int64)
    for i, (fr, fc) in enumerate(frontier):
        if rank[fr * 20 + fc] == _BIG:
            rank[fr * 20 + fc] = i
    cells = (r[:, None] + _DR[g]) * 20 + (c[:, None] + _DC[g])
    valid = np.arange(5)[None, :] < _NCELLS[g][:, None]
    cells = np.where(valid, np.clip(cells, 0, 399), 0)
    key = np.where(valid, rank[cells] * 8 + np.arange(5)[None, :], _BIG * 8)
    key = key.min(axis=1)
    order = np.lexsort((key, g))
    return g[order], r[order], c[order]


def frontier_ranks(sets: np.ndarray, players) -> np.ndarray:
    """rank[i, cell]: the position of `cell` (r * 20 + c) in the iteration order of player
    players[i]'s frontier set held in sets[i] (FSET_DTYPE, the CPython table: slot order
    of the keys >= 0 in slots 0..mask), _BIG where absent.  The vectorised equivalent of
    ranking fset_list(sets[i], players[i]) (engine/board.py:247-258 get_frontier)."""
    m = len(sets)
    pl = np.asarray(players, dtype=np.int64)
    keys = sets["key"][np.arange(m), pl].astype(np.int64)  # [m, 256]
    mask = sets["mask"][np.arange(m), pl].astype(np.int64)
    valid = (keys >= 0) & (np.arange(keys.shape[1])[None, :] <= mask[:, None])
    order = np.cumsum(valid, axis=1) - 1
    rank = np.full((m, 400), _BIG, dtype=np.int64)
    ii, ss = np.nonzero(valid)
    rank[ii, keys[ii, ss]] = order[ii, ss]  # a set holds each key once
    return rank


def order_moves_many(rows: np.ndarray, frontiers: Optional[Sequence[Sequence]] = None, *,
                     ranks: Optional[np.ndarray] = None):
    """order_moves for m board-players at once: rows uint32[m,91,20], frontiers[i] the
    iteration-order (row, col) list of board-player i's frontier set (or ranks, int64
    [m, 400], from frontier_ranks).  Returns a list of m (g, r, c) tuples, each in the
    reference's frontier list order (the key of order_moves: piece asc, orientation asc,
    min over the move's cells on a frontier cell of (rank, cell index))."""
    rows = np.ascontiguousarray(rows, dtype="<u4")
    m = rows.shape[0]
    if m == 0:
        return []
    # only the nonzero row words are unpacked (most of the 91 x 20 rows hold no anchor)
    gi, g, r = np.nonzero(rows)
    words = rows[gi, g, r]
    bits = np.unpackbits(words.view(np.uint8).reshape(-1, 4), axis=1, bitorder="little")
    w, c = np.nonzero(bits)  # word-major (game, g, r ascending), columns ascending
    gi, g, r = gi[w], g[w], r[w]
    rank = ranks
    if rank is None:
        rank = np.full((m, 400), _BIG, dtype=np.int64)
        for i, fr in enumerate(frontiers):
            for j, (a, b) in enumerate(fr):
                if rank[i, a * 20 + b] == _BIG:
                    rank[i, a * 20 + b] = j
    cells = (r[:, None] + _DR[g]) * 20 + (c[:, None] + _DC[g])
    valid = np.arange(5)[None, :] < _NCELLS[g][:, None]
    cells = np.where(valid, np.clip(cells, 0, 399), 0)
    key = np.where(valid, rank[gi[:, None], cells] * 8 + np.arange(5)[None, :], _BIG * 8).min(axis=1)
    order = np.lexsort((key, g, gi))
    gi, g, r, c = gi[order], g[order], r[order], c[order]
    cuts = np.searchsorted(gi, np.arange(1, m))
    return [(gg, rr, cc) for gg, rr, cc in zip(np.split(g, cuts), np.split(r, cuts), np.split(c, cuts))]


class LegalMoveGenerator:
    """Drop-in for engine.move_generator.LegalMoveGenerator, GPU-backed."""

    def __init__(self, device: int = 0):
        self.piece_generator = PieceGenerator()
        self.all_pieces = self.piece_generator.get_all_pieces()
        self.piece_orientations_cache = {}
        self.piece_position_cache = {}
        for piece in self.all_pieces:
            shapes = self.piece_generator.get_piece_rotations_and_reflections(piece)
            self.piece_orientations_cache[piece.id] = shapes
            self.piece_position_cache[piece.id] = [PiecePlacement.get_piece_positions(s, 0, 0) for s in shapes]
        self.device = device
        self._gpu = threading.local()

    # ------------------------------------------------------------------ GPU
    def _engine(self):
        eng = getattr(self._gpu, "engine", None)
        if eng is None:
            from ..gpu import BlokusGPU
            eng = BlokusGPU(self.device)  # raises NativeUnavailable without library/GPU
            self._gpu.engine = eng
        return eng

    @staticmethod
    def _legality_key(state) -> bytes:
        """The packed fields a legal set depends on: planes, used pieces, first-move flags."""
        return state["planes"].tobytes() + state["used"].tobytes() + state["first_move"].tobytes()

    def _masks(self, boards: Sequence[Board], players: Sequence[Player]):
        from .board import pack_states
        states = pack_states(boards)
        pl = np.array([p.value - 1 for p in players], dtype=np.uint8)
        if len(boards) == 1:  # the rows players_with_moves fetched for this very position
            last = getattr(self._gpu, "last_rows", None)
            if last is not None and last[0] == self._legality_key(states[0]):
                k = int(pl[0])
                return last[1][k:k + 1], last[2][k:k + 1]
        return self._engine().movegen(states, pl, rows=True)

    @staticmethod
    def _to_moves(g, r, c) -> List[Move]:
        return [Move(int(_PID[gi]), int(_OID[gi]), int(ri), int(ci)) for gi, ri, ci in zip(g, r, c)]

    # ------------------------------------------------------------------ API
    def get_legal_moves(self, board: Board, player: Player) -> List[Move]:
        if USE_FRONTIER_MOVEGEN:
            return self._get_legal_moves_frontier(board, player)
        return self._get_legal_moves_naive(board, player)

    def get_legal_moves_batch(self, boards: Sequence[Board], players: Sequence[Player],
                              order: str = "frontier" if USE_FRONTIER_MOVEGEN else "naive") -> List[List[Move]]:
        """One GPU launch for many (board, player) pairs."""
        if not boards:
            return []
        _, rows = self._masks(boards, players)
        out = []
        for i, (b, p) in enumerate(zip(boards, players)):
            fr = list(b.get_frontier(p)) if order == "frontier" else None
            out.append(self._to_moves(*order_moves(rows[i], fr)))
        return out

    def _get_legal_moves_naive(self, board: Board, player: Player) -> List[Move]:
        _, rows = self._masks([board], [player])
        return self._to_moves(*order_moves(rows[0], None))

    def _get_legal_moves_frontier(self, board: Board, player: Player) -> List[Move]:
        _, rows = self._masks([board], [player])
        return self._to_moves(*order_moves(rows[0], list(board.get_frontier(player))))

    def get_move_count(self, board: Board, player: Player) -> int:
        from .board import pack_states
        cnt, _ = self._engine().movegen(pack_states([board]), np.array([player.value - 1], np.uint8), rows=False)
        return int(cnt[0])

    def has_legal_moves(self, board: Board, player: Player) -> bool:
        return self.get_move_count(board, player) > 0

    def players_with_moves(self, board: Board) -> List[bool]:
        """has_legal_moves for all four players in ONE launch (BlokusGame._check_game_over).
        The launch also returns the four legal sets, kept (per thread, keyed by the packed
        position) for the next get_legal_moves on the same position -- the next player's
        turn in a game loop -- so a ply costs one launch, not two."""
        from .board import pack_states
        st = pack_states([board])
        cnt, rows = self._engine().movegen(np.repeat(st, 4), np.arange(4, dtype=np.uint8), rows=True)
        self._gpu.last_rows = (self._legality_key(st[0]), cnt, rows)
        return [int(c) > 0 for c in cnt]

    def _has_any_legal_move_frontier(self, board: Board, player: Player) -> bool:
        return self.has_legal_moves(board, player)

    def get_legal_moves_for_piece(self, board: Board, player: Player, piece_id: int) -> List[Move]:
        if piece_id in board.player_pieces_used[player]:
            return []
        _, rows = self._masks([board], [player])
        g, r, c = order_moves(rows[0], None)
        keep = _PID[g] == piece_id
        return self._to_moves(g[keep], r[keep], c[keep])

    # ------------------------------------------------------------- host checks
    def is_move_legal(self, board: Board, player: Player, move: Move) -> bool:
        """Single-move validation on the host (engine/move_generator.py:912-946)."""
        if move.piece_id in board.player_pieces_used[player]:
            return False
        shapes = self.piece_orientations_cache.get(move.piece_id, [])
        if not 0 <= move.orientation < len(shapes):
            return False
        shape = shapes[move.orientation]
        if not PiecePlacement.can_place_piece_at((board.SIZE, board.SIZE), shape, move.anchor_row, move.anchor_col):
            return False
        return board.can_place_piece(move.get_positions(shapes), player)

    def is_placement_legal_bitboard(self, board: Board, player: Player, orientation: PieceOrientation,
                                    anchor_board_coord, anchor_piece_index: int = 0) -> bool:
        """Anchor-cell legality (move_generator.py:561-655): offsets[anchor_piece_index] is put
        on anchor_board_coord; the shape is shifted with strict shift_mask (off-board -> False),
        neighbours are derived from the shifted cells, first-move status from the board."""
        if anchor_piece_index >= len(orientation.offsets):
            return False
        pr, pc = orientation.offsets[anchor_piece_index]
        shifted = shift_mask(orientation.shape_mask, anchor_board_coord[0] - pr, anchor_board_coord[1] - pc)
        if shifted is None:
            return False
        return self.is_placement_legal_bitboard_coords(
            board, player, mask_to_coords(shifted), is_first_move=board.player_first_move[player])

    def is_placement_legal_grid(self, board: Board, player: Player, orientation: PieceOrientation,
                                anchor_board_coord, anchor_piece_index: int, placement_coords) -> bool:
        """Grid legality of explicit cells (move_generator.py:657-680); orientation/anchor unused."""
        return board.can_place_piece([Position(r, c) for r, c in placement_coords], player)

    def is_placement_legal_bitboard_fast(self, board: Board, player: Player, piece_orientation: PieceOrientation,
                                         anchor_row: int, anchor_col: int, is_first_move: bool = False) -> bool:
        """Single-anchor legality from bitboards (move_generator.py:760-831)."""
        cells = [(anchor_row + r, anchor_col + c) for r, c in piece_orientation.offsets]
        return self.is_placement_legal_bitboard_coords(board, player, cells, is_first_move=is_first_move)

    def is_placement_legal_bitboard_coords(self, board: Board, player: Player, placement_coords,
                                           *, is_first_move: bool = False) -> bool:
        n = board.SIZE
        if any(not (0 <= r < n and 0 <= c < n) for r, c in placement_coords):
            return False
        shape = 0
        for r, c in placement_coords:
            shape |= BIT_TABLE[r][c]
        if shape & board.occupied_bits:
            return False
        own = board.player_bits[player]
        cs = set(placement_coords)
        diag = orth = 0
        for r, c in placement_coords:
            for dr, dc in ((-1, 0), (1, 0), (0, -1), (0, 1)):
                rr, cc = r + dr, c + dc
                if 0 <= rr < n and 0 <= cc < n and (rr, cc) not in cs:
                    orth |= BIT_TABLE[rr][cc]
            for dr, dc in ((-1, -1), (-1, 1), (1, -1), (1, 1)):
                rr, cc = r + dr, c + dc
                if 0 <= rr < n and 0 <= cc < n and (rr, cc) not in cs:
                    diag |= BIT_TABLE[rr][cc]
        if orth & own:
            return False
        if is_first_move:
            corner = board.player_start_corners[player]
            return bool(shape & BIT_TABLE[corner.row][corner.col])
        return bool(diag & own)

    def get_game_state_summary(self, board: Board) -> dict:
        return {
            "current_player": board.current_player, "move_count": board.move_count,
            "game_over": board.game_over,
            "player_moves": {p.name: self.get_move_count(board, p) for p in Player},
            "player_scores": {p.name: board.get_score(p) for p in Player},
            "player_pieces_used": {p.name: len(board.player_pieces_used[p]) for p in Player},
        }


_SHARED: Optional[LegalMoveGenerator] = None
_SHARED_LOCK = threading.Lock()


def get_shared_generator() -> LegalMoveGenerator:
    global _SHARED
    with _SHARED_LOCK:
        if _SHARED is None:
            _SHARED = LegalMoveGenerator()
    return _SHARED


def _neighbour_sets(cells):
    n = Board.SIZE
    placed = set(cells)
    diag, orth = set(), set()
    for r, c in cells:
        for (dr, dc), dst in (((-1, -1), diag), ((-1, 1), diag), ((1, -1), diag), ((1, 1), diag),
                              ((-1, 0), orth), ((1, 0), orth), ((0, -1), orth), ((0, 1), orth)):
            rr, cc = r + dr, c + dc
            if 0 <= rr < n and 0 <= cc < n and (rr, cc) not in placed:
                dst.add((rr, cc))
    return diag, orth


def debug_compare_bitboard_vs_grid(board: Board, player: Player, orientation: PieceOrientation,
                                   anchor_board_coord, anchor_piece_index: int, placement_coords) -> None:
    """Debug report (move_generator.py:1083-1217): masks from the explicit cells vs the
    orientation's precomputed masks shifted to the anchor, the overlap/adjacency hits, and
    grid vs bitboard legality.  Prints only when BLOKUS_DEBUG_BITBOARD is set."""
    if not DEBUG_BITBOARD:
        return
    diag_set, orth_set = _neighbour_sets(placement_coords)
    pr, pc = orientation.offsets[anchor_piece_index]
    d_row, d_col = anchor_board_coord[0] - pr, anchor_board_coord[1] - pc
    shifted = {k: shift_mask(getattr(orientation, k + "_mask"), d_row, d_col) for k in ("shape", "diag", "orth")}
    line = "=" * 80
    print("\n" + line)
    print("=== DEBUG BITBOARD VS GRID ===")
    print(f"player={player.name} (value={player.value})")
    print(f"piece_id={orientation.piece_id}")
    print(f"anchor_board_coord={anchor_board_coord}, anchor_piece_index={anchor_piece_index}")
    print(f"d_row={d_row}, d_col={d_col} (computed from board_r={anchor_board_coord[0]} - piece_r={pr}, "
          f"board_c={anchor_board_coord[1]} - piece_c={pc})")
    print(f"placement_coords={sorted(placement_coords)}")
    print()
    for title, a_label, a, b_label, key in (
            ("Shape from coords vs shifted shape:", "coords -> mask -> coords",
             sorted(mask_to_coords(coords_to_mask(placement_coords))), "shifted orientation shape coords", "shape"),
            ("Diag neighbors from coords vs shifted diag mask:", "diag from coords", sorted(diag_set),
             "diag mask coords", "diag"),
            ("Orth neighbors from coords vs shifted orth mask:", "orth from coords", sorted(orth_set),
             "orth mask coords", "orth")):
        b = sorted(mask_to_coords(shifted[key] or 0))
        print(title)
        print(f"  {a_label}: {a}")
        print(f"  {b_label}: {b}")
        print(f"  MATCH: {a == b}")
        print()
    own, occ = board.player_bits[player], board.occupied_bits
    hits = {"Overlap": (shifted["shape"] or 0) & occ, "Orth adj": (shifted["orth"] or 0) & own,
            "Diag adj": (shifted["diag"] or 0) & own}
    print("Adjacency & overlap checks:")
    print(f"  shape & occupied_bits -> {bool(hits['Overlap'])} (should be False for legal)")
    print(f"  orth & player_bits     -> {bool(hits['Orth adj'])} (should be False for legal)")
    print(f"  diag & player_bits      -> {bool(hits['Diag adj'])} (should be True if not first move)")
    print()
    for name, m in hits.items():
        if m:
            print(f"  {name} cells: {sorted(mask_to_coords(m))}")
    print()
    gen = LegalMoveGenerator()
    grid_legal = gen.is_placement_legal_grid(board, player, orientation, anchor_board_coord,
                                             anchor_piece_index, placement_coords)
    bit_legal = gen.is_placement_legal_bitboard(board, player, orientation, anchor_board_coord, anchor_piece_index)
    print(f"RESULT: grid_legal={grid_legal}, bitboard_legal={bit_legal}")
    if grid_legal != bit_legal:
        print("  *** MISMATCH DETECTED ***")
    print("=== END DEBUG ===")
    print(line)
    print()


def move_to_int(m: Move) -> int:
    """g * 400 + row * 20 + col (the Discrete(36400) action id)."""
    return GID[(m.piece_id, m.orientation)] * 400 + m.anchor_row * 20 + m.anchor_col


def int_to_move(a: int) -> Move:
    g, rest = divmod(int(a), 400)
    pid, o = ORIENT_LIST[g]
    return Move(pid, o, rest // 20, rest % 20)
