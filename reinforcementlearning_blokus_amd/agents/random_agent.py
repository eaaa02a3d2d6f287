"""Uniform random policy (reference: agents/random_agent.py:14-66).

numpy RandomState(seed).randint(0, len(legal)) -- MT19937 with legacy masked
rejection; a one-element list consumes no draw.  The GPU rollout kernel's compat
stream (BK_RNG_NUMPY_MT) reproduces exactly this sequence.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional

import numpy as np

from ..engine.board import Board, Player
from ..engine.move_generator import Move, get_shared_generator
from ..engine.pieces import PieceGenerator


class RandomAgent:
    def __init__(self, seed: Optional[int] = None):
        self.seed = seed
        self.rng = np.random.RandomState(seed)
        self.move_generator = get_shared_generator()
        self.piece_generator = PieceGenerator()

    def select_action(self, board: Board, player: Player, legal_moves: List[Move]) -> Optional[Move]:
        if not legal_moves:
            return None
        return legal_moves[self.rng.randint(0, len(legal_moves))]

    def get_action_info(self) -> Dict[str, Any]:
        return {"name": "RandomAgent", "type": "random", "description": "Selects moves uniformly from legal actions"}

    def reset(self):
        pass

    def set_seed(self, seed: int):
        self.seed = seed
        self.rng = np.random.RandomState(seed)
