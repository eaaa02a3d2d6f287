"""Heuristic policy (reference: agents/heuristic_agent.py:14-244).

Every legal move is scored as in the reference's ``_evaluate_move`` (:68-105):

    score = 0.0 + w_size * piece size
                + w_corner * corner creation   (:107-138)
                + w_edge * edge avoidance      (:140-176)
                + w_center * centre preference (:178-199)

then a softmax (:223-244) turns the scores into probabilities and
``RandomState(seed).choice`` draws the move (:61-65).

The scores of a whole legal list are computed at once from board bitmaps (numpy),
with the reference's float64 operations in the reference's order, so they are the
same doubles as its per-move Python evaluation (pinned by tests/golden/heuristic.json):

* corner creation of a placement = sum over its cells of D(cell), where D(cell) counts
  the cell's in-bounds diagonal neighbours that are empty and have no orthogonal
  neighbour owned by the mover on the board BEFORE the move -- exactly the
  reference's nested loop (a neighbour reached from two cells counts twice);
* edge avoidance = cells with min(r, c, 19 - r, 19 - c) <= 2, halved from move 30 on
  (``move_count / 100.0 < 0.3``);
* centre preference = 1 - |anchor - (9.5, 9.5)| / sqrt(2 * 9.5**2).

The softmax and the draw use numpy itself (``np.exp``, ``np.sum``,
``RandomState.choice``), so the chosen move is the reference's for the same seed.
The legal list (and its order) comes from the GPU move generator.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional

import numpy as np

from ..engine.board import Board, Player, Position
from ..engine.move_generator import Move, get_shared_generator
from ..engine.pieces import GID, ORIENT_CELLS, PieceGenerator

_NC = np.array([len(c) for c in ORIENT_CELLS], dtype=np.int64)
_DR = np.zeros((len(ORIENT_CELLS), 5), dtype=np.int64)
_DC = np.zeros((len(ORIENT_CELLS), 5), dtype=np.int64)
for _g, _cells in enumerate(ORIENT_CELLS):
    for _k, (_r, _c) in enumerate(_cells):
        _DR[_g, _k], _DC[_g, _k] = _r, _c
_VALID = np.arange(5)[None, :] < _NC[:, None]

_R, _C = np.meshgrid(np.arange(20), np.arange(20), indexing="ij")
_NEAR_EDGE = (np.minimum(np.minimum(_R, _C), np.minimum(19 - _R, 19 - _C)) <= 2).astype(np.int64).reshape(-1)
_MAX_DISTANCE = np.sqrt(2 * (9.5 ** 2))


def corner_map(grid: np.ndarray, player_value: int) -> np.ndarray:
    """D[r, c] (int, 0..4): in-bounds diagonal neighbours of (r, c) that are empty and
    not orthogonally adjacent to ``player_value`` (heuristic_agent.py:120-136)."""
    own = np.pad(grid == player_value, 1)
    orth = own[:-2, 1:-1] | own[2:, 1:-1] | own[1:-1, :-2] | own[1:-1, 2:]
    safe = np.pad((grid == 0) & ~orth, 1).astype(np.int64)
    return safe[:-2, :-2] + safe[:-2, 2:] + safe[2:, :-2] + safe[2:, 2:]


def score_moves(board: Board, player: Player, gids: np.ndarray, ar: np.ndarray, ac: np.ndarray,
                weights=(1.0, 2.0, -1.5, 0.5)) -> np.ndarray:
    """_evaluate_move for many placements at once: orientation ids (global), anchors ->
    float64 scores, bit-identical to the reference's per-move evaluation."""
    w_size, w_corner, w_edge, w_center = weights
    gids = np.asarray(gids, dtype=np.int64)
    ar = np.asarray(ar, dtype=np.int64)
    ac = np.asarray(ac, dtype=np.int64)
    valid = _VALID[gids]
    cells = np.where(valid, (ar[:, None] + _DR[gids]) * 20 + ac[:, None] + _DC[gids], 0)
    d = corner_map(board.grid, player.value).reshape(-1)
    corner = np.where(valid, d[cells], 0).sum(axis=1)
    edge = np.where(valid, _NEAR_EDGE[cells], 0).sum(axis=1)
    size = _NC[gids]
    if board.move_count / 100.0 < 0.3:
        edge_score = edge
    else:
        edge_score = edge * 0.5
    distance = np.sqrt((ar - 9.5) ** 2 + (ac - 9.5) ** 2)
    center = 1.0 - distance / _MAX_DISTANCE
    score = 0.0 + w_size * size
    score = score + w_corner * corner
    score = score + w_edge * edge_score
    score = score + w_center * center
    return np.asarray(score, dtype=np.float64)


class HeuristicAgent:
    """Drop-in for agents.heuristic_agent.HeuristicAgent."""

    def __init__(self, seed: Optional[int] = None):
        self.rng = np.random.RandomState(seed)
        self.move_generator = get_shared_generator()
        self.piece_generator = PieceGenerator()
        self.piece_size_weight = 1.0
        self.corner_creation_weight = 2.0
        self.edge_avoidance_weight = -1.5
        self.center_preference_weight = 0.5

    def _weights(self):
        return (self.piece_size_weight, self.corner_creation_weight, self.edge_avoidance_weight,
                self.center_preference_weight)

    def score_legal_moves(self, board: Board, player: Player, legal_moves: List[Move]) -> np.ndarray:
        """Scores of a whole legal list (reference: one _evaluate_move per move)."""
        gids = np.fromiter((GID[(m.piece_id, m.orientation)] for m in legal_moves), dtype=np.int64,
                           count=len(legal_moves))
        ar = np.fromiter((m.anchor_row for m in legal_moves), dtype=np.int64, count=len(legal_moves))
        ac = np.fromiter((m.anchor_col for m in legal_moves), dtype=np.int64, count=len(legal_moves))
        return score_moves(board, player, gids, ar, ac, self._weights())

    def select_action(self, board: Board, player: Player, legal_moves: List[Move]) -> Optional[Move]:
        if not legal_moves:
            return None
        probabilities = self._softmax(self.score_legal_moves(board, player, legal_moves), temperature=1.0)
        move_idx = self.rng.choice(len(legal_moves), p=probabilities)
        return legal_moves[move_idx]

    def _evaluate_move(self, board: Board, player: Player, move: Move) -> float:
        return float(self.score_legal_moves(board, player, [move])[0])

    def _get_piece_positions(self, move: Move, orientation: np.ndarray) -> List[Position]:
        rows, cols = orientation.shape
        return [Position(move.anchor_row + i, move.anchor_col + j)
                for i in range(rows) for j in range(cols) if orientation[i, j] == 1]

    def _softmax(self, x: np.ndarray, temperature: float = 1.0) -> np.ndarray:
        x_scaled = x / temperature
        x_max = np.max(x_scaled)
        x_shifted = x_scaled - x_max
        exp_x = np.exp(x_shifted)
        return exp_x / np.sum(exp_x)

    def get_action_info(self) -> Dict[str, Any]:
        return {"name": "HeuristicAgent", "type": "heuristic",
                "description": "Strategic agent with piece size, corner, and edge preferences",
                "weights": {"piece_size": self.piece_size_weight, "corner_creation": self.corner_creation_weight,
                            "edge_avoidance": self.edge_avoidance_weight,
                            "center_preference": self.center_preference_weight}}

    def reset(self):
        pass

    def set_seed(self, seed: int):
        self.rng = np.random.RandomState(seed)

    def set_weights(self, weights: Dict[str, float]):
        if "piece_size" in weights:
            self.piece_size_weight = weights["piece_size"]
        if "corner_creation" in weights:
            self.corner_creation_weight = weights["corner_creation"]
        if "edge_avoidance" in weights:
            self.edge_avoidance_weight = weights["edge_avoidance"]
        if "center_preference" in weights:
            self.center_preference_weight = weights["center_preference"]
