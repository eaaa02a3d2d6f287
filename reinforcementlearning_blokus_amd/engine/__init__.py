"""Drop-in mirror of the reference ``engine`` package (engine/__init__.py:12-22)."""
from .board import Board, Player, Position
from .game import BlokusGame, GameResult
from .move_generator import LegalMoveGenerator, Move, get_shared_generator
from .pieces import Piece, PieceGenerator, PiecePlacement, PieceType

__all__ = ["Board", "Player", "Position", "Piece", "PieceType", "PieceGenerator", "PiecePlacement",
           "Move", "LegalMoveGenerator", "BlokusGame", "GameResult", "get_shared_generator"]
