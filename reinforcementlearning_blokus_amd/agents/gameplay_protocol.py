"""Web-runtime agent contract (reference: agents/gameplay_protocol.py:13-25)."""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Protocol, Tuple

from ..engine.board import Board, Player
from ..engine.move_generator import Move


class GameplayAgentProtocol(Protocol):
    def choose_move(self, board: Board, player: Player, legal_moves: List[Move],
                    time_budget_ms: int) -> Tuple[Optional[Move], Dict[str, Any]]:
        ...
