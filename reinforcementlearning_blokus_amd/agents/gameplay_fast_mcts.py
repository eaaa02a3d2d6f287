"""choose_move() adapter over FastMCTSAgent (reference: agents/gameplay_fast_mcts.py:14-37)."""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple

from ..engine.board import Board, Player
from ..engine.move_generator import Move
from .fast_mcts_agent import FastMCTSAgent


class GameplayFastMCTSAgent:
    def __init__(self, *, iterations: int = 5000, exploration_constant: float = 1.414,
                 seed: Optional[int] = None, device: int = 0) -> None:
        self._agent = FastMCTSAgent(iterations=iterations, time_limit=1.0,
                                    exploration_constant=exploration_constant, seed=seed, device=device)

    def choose_move(self, board: Board, player: Player, legal_moves: List[Move],
                    time_budget_ms: int) -> Tuple[Optional[Move], Dict[str, Any]]:
        result = self._agent.think(board, player, legal_moves, time_budget_ms)
        return result.get("move"), dict(result.get("stats") or {})
