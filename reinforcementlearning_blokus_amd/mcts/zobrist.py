"""Zobrist hashing + transposition table (reference: mcts/zobrist.py:12-220).

Keys are numpy RandomState(seed).randint(0, 2**64, dtype=uint64) draws in the
reference's order (cell x value, then turn, then player x piece), so hashes are
bit-identical to the reference's for the same seed (pinned by tests/golden/zobrist.json).
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

from ..engine.board import Board, Player


class ZobristHash:
    def __init__(self, board_size: int = 20, num_players: int = 4, seed: Optional[int] = None):
        self.board_size = board_size
        self.num_players = num_players
        self.rng = np.random.RandomState(seed)
        self._generate_hash_values()

    def _generate_hash_values(self):
        # the reference draws one randint(0, 2**64, dtype=uint64) per key, cell x value,
        # then turn, then player x piece (mcts/zobrist.py:41-68); a full-range uint64 draw
        # is next_uint64 per element whether drawn one at a time or as one array, so one
        # vector draw in that order gives the same keys (tests/golden/zobrist.json)
        n, k = self.board_size, self.num_players
        vals = self.rng.randint(0, 2**64, size=n * n * (k + 1) + k + k * 21, dtype=np.uint64)
        m = n * n * (k + 1)
        self.position_player_hashes = vals[:m].reshape(n, n, k + 1).copy()
        self.player_turn_hashes = vals[m:m + k].copy()
        self.piece_used_hashes = vals[m + k:].reshape(k, 21).copy()
        # flat view used for vectorised hashing: index cell * (k+1) + value
        self._flat = self.position_player_hashes.reshape(-1)

    def hash_board(self, board: Board) -> int:
        idx = np.arange(self.board_size * self.board_size) * (self.num_players + 1) + board.grid.reshape(-1)
        h = np.bitwise_xor.reduce(self._flat[idx])
        h ^= self.player_turn_hashes[board.current_player.value - 1]
        for p in Player:
            for pid in board.player_pieces_used[p]:
                h ^= self.piece_used_hashes[p.value - 1, pid - 1]
        return np.uint64(h)

    def hash_move(self, board: Board, move_hash: int, player: Player, piece_id: int) -> int:
        i = board.current_player.value - 1
        h = np.uint64(move_hash) ^ self.player_turn_hashes[i] ^ self.player_turn_hashes[(i + 1) % self.num_players]
        return h ^ self.piece_used_hashes[player.value - 1, piece_id - 1]

    def hash_position_placement(self, row: int, col: int, player: Player) -> int:
        return self.position_player_hashes[row, col, player.value]

    def get_hash_info(self):
        return {"board_size": self.board_size, "num_players": self.num_players, "hash_bits": 64,
                "total_positions": self.board_size * self.board_size, "total_pieces": 21}


class TranspositionTable:
    def __init__(self, max_size: int = 1000000):
        self.max_size = max_size
        self.table: Dict[int, Dict] = {}
        self.access_count = 0
        self.hit_count = 0
        self.gpu_size = 0  # entries held in the GPU search backend's device-layout table

    def get(self, hash_value: int) -> Optional[Dict]:
        self.access_count += 1
        e = self.table.get(hash_value)
        if e is not None:
            self.hit_count += 1
        return e

    def put(self, hash_value: int, entry: Dict):
        if len(self.table) >= self.max_size:
            for key in list(self.table.keys())[: self.max_size // 10]:
                del self.table[key]
        self.table[hash_value] = entry

    def clear(self):
        self.table.clear()
        self.gpu_size = 0
        self.access_count = 0
        self.hit_count = 0

    def get_stats(self) -> Dict[str, float]:
        return {"size": len(self.table) + self.gpu_size, "max_size": self.max_size, "access_count": self.access_count,
                "hit_count": self.hit_count, "hit_rate": self.hit_count / max(self.access_count, 1)}


def flat_keys(z: ZobristHash) -> np.ndarray:
    """The 2088-word key table bk_mcts reads: cells x 5 values (row-major, value
    0 = empty, p = player p), 4 turn keys, 4 x 21 piece keys (mcts/zobrist.py:41-68)."""
    return np.concatenate([z.position_player_hashes.reshape(-1), z.player_turn_hashes,
                           z.piece_used_hashes.reshape(-1)]).astype(np.uint64)


def hash_states(states: np.ndarray, keys: np.ndarray) -> np.ndarray:
    """ZobristHash.hash_board (mcts/zobrist.py:70-99) of packed bk_state records,
    vectorised: XOR of the 400 cell keys, the side-to-move key and the used-piece keys.
    keys: one 2088-word table (flat_keys) for every state, or one table per state
    ([n, 2088])."""
    states = np.atleast_1d(states)
    keys = np.asarray(keys, dtype=np.uint64)
    per_state = keys.ndim == 2 and keys.shape[0] == len(states) and keys.shape[1] == 2088
    if not per_state:
        keys = keys.reshape(-1)
    n = len(states)
    if n == 0:  # (a rank's shard may hold no game of some table: games r mod W, tables i mod 8)
        return np.zeros(0, np.uint64)
    cells = np.arange(400)
    word, bit = cells // 64, (cells % 64).astype(np.uint64)
    grid = np.zeros((n, 400), np.int64)
    for p in range(4):
        occ = (states["planes"][:, p, word] >> bit) & np.uint64(1)
        grid += occ.astype(np.int64) * (p + 1)
    # used-piece keys: [n, 4, 21] on/off
    used = states["used"].astype(np.int64)  # [n, 4]
    pidx = 2004 + np.arange(4)[:, None] * 21 + np.arange(21)[None, :]  # [4, 21]
    pon = ((used[:, :, None] >> np.arange(21)[None, None, :]) & 1) == 1  # [n, 4, 21]
    if per_state:
        cellk = np.take_along_axis(keys, cells * 5 + grid, axis=1)
        h = np.bitwise_xor.reduce(cellk, axis=1)
        h ^= keys[np.arange(n), 2000 + states["current_player"].astype(np.int64)]
        pk = np.where(pon, keys[:, pidx.reshape(-1)].reshape(n, 4, 21), np.uint64(0))
    else:
        h = np.bitwise_xor.reduce(keys[cells * 5 + grid], axis=1)
        h ^= keys[2000 + states["current_player"].astype(np.int64)]
        pk = np.where(pon, keys[pidx][None, :, :], np.uint64(0))
    h ^= np.bitwise_xor.reduce(pk.reshape(n, -1), axis=1)
    return h.astype(np.uint64)
