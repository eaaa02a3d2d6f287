"""BASELINE.json workloads on the GPU, shared by bench.py and the -m gpu tests.

Config 5 (BASELINE.json configs[4]): 65,536 concurrent games, each searching its
position with MCTSAgent (mcts/mcts_agent.py:304-582, RandomAgent rollouts, Zobrist
transposition table, mcts/zobrist.py:12-220) for 4,096 iterations, every tree, TT and
RNG stream resident in HBM (bk_mcts, BK_MEM_DEVICE).
"""
from __future__ import annotations

import numpy as np

from . import _native as N
from .gpu import BlokusGPU, empty_state, mcts_log_table, mcts_node_cap


def frontier_roots(gpu: BlokusGPU, n: int, plies: int, seed: int, *, distinct: int | None = None,
                   stream_base: int = 0):
    """n synthetic mid-game positions with their frontier-set tables: `plies` uniform
    random moves from the empty board in the reference's frontier list order (Philox
    stream (seed, stream_base + i) for position i), i.e. positions a reference Board
    reaches by place_piece.  distinct: make only that many positions and repeat them
    (position i % distinct)."""
    k = n if distinct is None else min(n, distinct)
    st, fs = gpu.rollout_frontier(empty_state(), N.fset_new(1), k, semantics=N.SEM_ADVANCE, rng=N.RNG_PHILOX,
                                  seed=seed, max_plies=plies, root_index=np.zeros(k, dtype=np.int32),
                                  stream_base=stream_base)
    if k < n:
        idx = np.arange(n) % k
        st, fs = st[idx], fs[idx]
    return st, fs


class Config3Plan:
    """Config 3's random streams as functions of the GLOBAL game index (BASELINE.json
    configs[2], weak scaling): rank r of a job plays global games r * games .. (r + 1) *
    games - 1, so the records an N-rank job gathers equal a 1-rank run of the same N *
    games games (per-game seeds are a pure function of (run seed, game
    index), analytics/tournament/arena_runner.py:248-254).

    * Root of global game G: `root_plies` uniform random moves from the empty board on
      Philox stream (seed, G) (bk_advance, or bk_rollout_frontier SEM_ADVANCE in frontier
      order).
    * Playout i of global game G (i < rollouts): global playout id P = G * rollouts + i,
      Philox stream (step_seed(k), P) in step k.
    A rank's launch uses its local ids with stream_base = the global id of its first."""

    def __init__(self, seed: int, games: int, rollouts: int, rank: int = 0):
        self.seed, self.games, self.rollouts, self.rank = int(seed), int(games), int(rollouts), int(rank)
        self.first_game = self.rank * self.games
        self.n_playouts = self.games * self.rollouts
        self.root_stream_base = self.first_game
        self.playout_stream_base = self.first_game * self.rollouts

    def step_seed(self, k: int) -> int:
        """Philox key of step k (warmup steps k = 0.., timed steps 1000 + k)."""
        return self.seed * 7919 + k

    def root_index(self) -> np.ndarray:
        """Local root of each local playout (a game's rollouts are contiguous: one wave
        plays 64 rollouts of the same game)."""
        return (np.arange(self.n_playouts, dtype=np.int64) // self.rollouts).astype(np.int32)

    def global_playouts(self) -> np.ndarray:
        return np.arange(self.n_playouts, dtype=np.int64) + self.playout_stream_base


def numpy_mt_states(seeds) -> np.ndarray:
    """uint32[n, 625]: numpy RandomState(seed) MT19937 key + pos per seed (the rollout
    agent's stream, agents/random_agent.py:29)."""
    from .mt19937 import seed_states
    seeds = np.asarray([int(s) for s in seeds], dtype=np.int64)
    out = np.zeros((len(seeds), 625), np.uint32)
    out[:, :624] = seed_states(seeds)  # (RandomState(seed) for all seeds at once)
    out[:, 624] = 624
    return out


def mcts_game_inputs(index, seed0: int = 0, n_tables: int = 8):
    """Per-game search inputs of global games `index` (a rank's shard or the whole job):
    zobrist table index i % n_tables (ZobristHash(seed=table), mcts/zobrist.py:41-68) and
    the rollout RandomAgent's MT19937 state for seed seed0 + i (agents/random_agent.py:29).
    Pure functions of the global index, so a sharded job searches exactly what one
    process would."""
    index = np.asarray(index, dtype=np.int64)
    zi = (index % n_tables).astype(np.int32)
    return zi, numpy_mt_states(seed0 + int(g) for g in index)


class MctsBatch:
    """Device-resident inputs and outputs of one bk_mcts batch (config 5 layout).

    Game g (global index i = index[g]) searches roots[g] for its player to move, with
    zobrist table i % n_tables (ZobristHash(seed=table), mcts/zobrist.py:41-68) and a
    rollout RandomAgent seeded seed0 + i.  Each game has its own TT of tt_cap slots (<= half full after
    `iterations` inserts) and a node pool of 4 * iterations + 1 slots."""

    def __init__(self, gpu: BlokusGPU, roots: np.ndarray, sets: np.ndarray, *, iterations: int, seed0: int = 0,
                 n_tables: int = 8, use_tt: bool = True, want_rewards: bool = False, max_rollout_moves: int = 50,
                 index=None):
        import torch

        from .mcts.zobrist import ZobristHash, flat_keys, hash_states
        self.gpu, self.iterations, self.max_rollout_moves = gpu, int(iterations), int(max_rollout_moves)
        dev = torch.device("cuda", gpu.device)
        n = self.n = len(roots)
        self.roots_np, self.sets_np = roots, sets
        self.players_np = np.asarray(roots["current_player"], np.uint8) & 3
        zob = np.stack([flat_keys(ZobristHash(seed=t)) for t in range(n_tables)])
        # global game indices (a rank's shard of a multi-GPU job): seeds and tables follow them
        self.index = np.arange(n) if index is None else np.asarray(index, dtype=np.int64)
        assert len(self.index) == n
        zi, self.mt0 = mcts_game_inputs(self.index, seed0, n_tables)
        rh = np.zeros(n, np.uint64)
        for t in range(n_tables):
            sel = zi == t
            rh[sel] = hash_states(roots[sel], zob[t])
        self.zobrist_np, self.zidx_np, self.hash_np = zob, zi, rh
        u8 = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(n, -1)).to(dev)  # noqa: E731
        self.roots, self.sets = u8(roots), u8(sets)
        self.players = torch.from_numpy(self.players_np.copy()).to(dev)
        self.root_hash = torch.from_numpy(rh.view(np.int64).copy()).to(dev)
        self.zobrist = torch.from_numpy(zob.view(np.int64).copy()).to(dev)
        self.zidx = torch.from_numpy(zi).to(dev)
        self.log_table = torch.from_numpy(mcts_log_table(self.iterations)).to(dev)
        self.node_cap = mcts_node_cap(self.iterations)
        self.nodes = torch.empty((n, self.node_cap * N.MCTS_NODE_DTYPE.itemsize), dtype=torch.uint8, device=dev)
        self.out = torch.zeros((n, N.MCTS_OUT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
        self.mt = torch.empty((n, 625), dtype=torch.int32, device=dev)
        self.tt_cap = 1 << max(1, int(np.ceil(np.log2(2 * (self.iterations + 1)))))
        if use_tt:
            self.tt_keys = torch.zeros((n, self.tt_cap), dtype=torch.int64, device=dev)
            self.tt_vals = torch.empty((n, self.tt_cap), dtype=torch.float64, device=dev)
            self.tt_count = torch.zeros(n, dtype=torch.int32, device=dev)
        else:
            self.tt_keys = self.tt_vals = self.tt_count = None
        if want_rewards:
            self.rewards = torch.zeros((n, self.iterations), dtype=torch.float64, device=dev)
            self.hit_flags = torch.zeros((n, self.iterations), dtype=torch.uint8, device=dev)
        else:
            self.rewards = self.hit_flags = None
        self.reset()

    def reset(self):
        """Fresh searches: RNG streams at their seeds, empty TTs."""
        import torch
        self.mt.copy_(torch.from_numpy(self.mt0.view(np.int32)))
        if self.tt_vals is not None:
            self.tt_vals.fill_(float("nan"))
            self.tt_count.zero_()

    def run(self, chunk: int = 0, on_chunk=None, stop_after: int | None = None,
            rollout_policy: int = N.MCTS_ROLLOUT_RANDOM):
        """Run the searches (launches of `chunk` iterations); stop_after: only the
        first stop_after iterations (a warm-up)."""
        self.gpu.mcts_device(self.roots, self.sets, self.players, self.root_hash, self.zobrist, self.zidx, self.mt,
                             self.log_table, self.nodes, self.out, iterations=self.iterations,
                             tt_keys=self.tt_keys, tt_vals=self.tt_vals, tt_count=self.tt_count,
                             rewards=self.rewards, hit_flags=self.hit_flags,
                             max_rollout_moves=self.max_rollout_moves, chunk=chunk, on_chunk=on_chunk,
                             stop_after=stop_after, rollout_policy=rollout_policy)

    def results(self) -> np.ndarray:
        return self.out.cpu().numpy().view(N.MCTS_OUT_DTYPE).reshape(-1)

    def root_children(self, g: int):
        """[(move, visits, total)] of game g's root children in expansion order."""
        root = self.nodes[g, :N.MCTS_NODE_DTYPE.itemsize].cpu().numpy().view(N.MCTS_NODE_DTYPE)[0]
        k, c0 = int(root["n_exp"]), int(root["child0"])
        isz = N.MCTS_NODE_DTYPE.itemsize
        blk = self.nodes[g, c0 * isz:(c0 + k) * isz].cpu().numpy().view(N.MCTS_NODE_DTYPE) if k else []
        return [(int(x["move"]), int(x["visits"]), float(x["total"])) for x in blk]
