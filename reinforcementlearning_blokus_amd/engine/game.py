"""BlokusGame on top of the GPU move generator (reference: engine/game.py).

Scoring, game-over and result semantics follow engine/game.py:57-349.  The
reference's per-move telemetry (engine/telemetry.py, ~80x the cost of a move) is UI
analytics outside the hot path: ``enable_telemetry`` is accepted and ignored.
``move_generator.has_legal_moves`` is looked up on the instance each time, so tests
can patch it exactly as the reference's tests do (tests/test_game_over_logic.py:31).
"""
from __future__ import annotations

import logging
from dataclasses import dataclass
from typing import Dict, List, Optional

from .board import Board, Player, Position
from .move_generator import LegalMoveGenerator, Move, get_shared_generator
from .pieces import PieceGenerator

logger = logging.getLogger(__name__)

_CORNERS = ((0, 0), (0, 19), (19, 0), (19, 19))
_CENTRE = [(r, c) for r in range(8, 12) for c in range(8, 12)]


@dataclass
class GameResult:
    scores: Dict[int, int]
    winner_ids: List[int]
    is_tie: bool


def _piece_penalty(used) -> int:
    """History metric only (engine/advanced_metrics.py:56-66 compute_piece_penalty):
    5 per unplayed U/W/X, 2 per other unplayed pentomino, 1 per unplayed tetromino."""
    pen = 0
    for pid in range(1, 22):
        if pid in used:
            continue
        pen += 5 if pid in (17, 19, 20) else 2 if pid >= 11 else 1 if pid >= 5 else 0
    return pen


class BlokusGame:
    def __init__(self, enable_telemetry: bool = True, telemetry_fast_mode: bool = True):
        self.board = Board()
        self.move_generator: LegalMoveGenerator = get_shared_generator()
        self.piece_generator = PieceGenerator()
        self.game_history = []
        self.winner = None
        self.enable_telemetry = enable_telemetry  # accepted; telemetry is out of scope
        self.telemetry_fast_mode = telemetry_fast_mode

    def make_move(self, move: Move, player: Optional[Player] = None) -> bool:
        """Validate, place, record, then check game over.  Illegal -> False."""
        if player is None:
            player = self.board.current_player
        if not self.move_generator.is_move_legal(self.board, player, move):
            return False
        rel = self.move_generator.piece_position_cache[move.piece_id][move.orientation]
        cells = [Position(move.anchor_row + r, move.anchor_col + c) for r, c in rel]
        ok = self.board.place_piece(cells, player, move.piece_id, validate=False)
        if ok:
            idx = len(self.game_history)
            sizes = {p.name: len(self.board.get_frontier(p)) for p in Player}
            self.game_history.append({
                "turn_number": idx + 1, "move_index": idx, "round_index": idx // 4,
                "position_in_round": idx % 4, "seat_index": player.value - 1,
                "player_to_move": player.name,
                "action": {"piece_id": move.piece_id, "orientation": move.orientation,
                           "anchor_row": move.anchor_row, "anchor_col": move.anchor_col},
                "board_state": self.board.grid.tolist(),
                "metrics": {"corner_count": dict(sizes), "frontier_size": dict(sizes),
                            "difficult_piece_penalty": {p.name: _piece_penalty(self.board.player_pieces_used[p])
                                                        for p in Player},
                            "remaining_pieces": {p.name: [i for i in range(1, 22)
                                                          if i not in self.board.player_pieces_used[p]]
                                                 for p in Player},
                            "influence_map": None},
            })
            self._check_game_over()
        return ok

    def _check_game_over(self) -> None:
        """Over iff no player has a legal move (engine/game.py:182-214)."""
        mg = self.move_generator
        batched = ("has_legal_moves" not in vars(mg) and hasattr(mg, "players_with_moves")
                   and getattr(type(mg), "has_legal_moves", None) is LegalMoveGenerator.has_legal_moves)
        if batched:  # one launch for the four players; a patched has_legal_moves is honoured
            if any(mg.players_with_moves(self.board)):
                return
        elif any(mg.has_legal_moves(self.board, p) for p in Player):
            return
        self.board.game_over = True
        res = self.get_game_result()
        self.winner = None if res.is_tie else Player(res.winner_ids[0])

    def get_game_result(self) -> GameResult:
        scores = {p.value: self.get_score(p) for p in Player}
        best = max(scores.values())
        winners = [pid for pid, s in scores.items() if s == best]
        return GameResult(scores=scores, winner_ids=winners, is_tie=len(winners) > 1)

    def get_winner(self) -> Optional[Player]:
        if not self.board.game_over:
            return None
        res = self.get_game_result()
        return None if res.is_tie else Player(res.winner_ids[0])

    def get_score(self, player: Player) -> int:
        return self.board.get_score(player) + self._calculate_bonus_score(player)

    def _calculate_bonus_score(self, player: Player) -> int:
        return self._calculate_corner_bonus(player) + self._calculate_center_bonus(player)

    def _calculate_corner_bonus(self, player: Player) -> int:
        return 5 * sum(int(self.board.grid[r, c] == player.value) for r, c in _CORNERS)

    def _calculate_center_bonus(self, player: Player) -> int:
        return 2 * sum(int(self.board.grid[r, c] == player.value) for r, c in _CENTRE)

    def get_legal_moves(self, player: Optional[Player] = None) -> List[Move]:
        return self.move_generator.get_legal_moves(self.board, player or self.board.current_player)

    def get_game_state(self) -> Dict:
        return {"board": self.board, "current_player": self.board.current_player,
                "move_count": self.board.move_count, "game_over": self.board.game_over,
                "winner": self.winner, "scores": {p.name: self.get_score(p) for p in Player},
                "legal_moves": len(self.get_legal_moves()), "game_history_length": len(self.game_history)}

    def reset_game(self) -> None:
        self.board = Board()
        self.game_history = []
        self.winner = None

    def get_board_copy(self) -> Board:
        return self.board.copy()

    def is_game_over(self) -> bool:
        return self.board.game_over

    def get_current_player(self) -> Player:
        return self.board.current_player

    def get_move_count(self) -> int:
        return self.board.move_count

    @property
    def move_count(self) -> int:
        return self.board.move_count

    def get_player_pieces_used(self, player: Player) -> int:
        return len(self.board.player_pieces_used[player])

    def get_player_pieces_remaining(self, player: Player) -> int:
        return 21 - self.get_player_pieces_used(player)

    def can_player_move(self, player: Player) -> bool:
        return self.move_generator.has_legal_moves(self.board, player)
