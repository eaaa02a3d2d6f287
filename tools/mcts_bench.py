#!/usr/bin/env python3
"""bk_mcts throughput: MCTSAgent searches (UCT + Zobrist TT + RandomAgent rollouts,
reference-exact) for G concurrent games from GPU-generated 20-ply positions.

Prints one JSON line per (games, iterations): searches, simulations (= iterations:
each one ends in a rollout or a TT hit), rollout plies are not counted; kernel time
from HIP events around the k_mcts launch, wall time including host staging.
Config 5 of BASELINE.json (65,536 games x 4,096 iterations) is the scale target."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, nargs="+", default=[4096])
    ap.add_argument("--iterations", type=int, nargs="+", default=[64])
    ap.add_argument("--max-rollout-moves", type=int, default=50)
    ap.add_argument("--no-tt", action="store_true")
    ap.add_argument("--seed", type=int, default=7)
    args = ap.parse_args()
    from reinforcementlearning_blokus_amd import _native as N
    from reinforcementlearning_blokus_amd.gpu import BlokusGPU, MctsTT, empty_state
    from reinforcementlearning_blokus_amd.mcts.zobrist import ZobristHash, flat_keys, hash_states
    gpu = BlokusGPU(0)
    keys = flat_keys(ZobristHash(seed=args.seed))
    for G in args.games:
        roots, sets = gpu.rollout_frontier(empty_state(), N.fset_new(1), G, semantics=N.SEM_ADVANCE,
                                           rng=N.RNG_PHILOX, seed=args.seed, max_plies=20,
                                           root_index=np.zeros(G, dtype=np.int32))
        players = roots["current_player"].copy()
        rh = hash_states(roots, keys)
        mt0 = np.zeros((G, 625), np.uint32)
        for g in range(G):
            st = np.random.RandomState(1000 + g).get_state()
            mt0[g, :624], mt0[g, 624] = st[1], st[2]
        for it in args.iterations:
            mt = mt0.copy()
            cap = 8
            while cap < 2 * (it + 2):
                cap *= 2
            tt = None if args.no_tt else MctsTT(G, cap=cap)
            t0 = time.perf_counter()
            r = gpu.mcts(roots, sets, players, rh, iterations=it, zobrist=keys[None], mt_state=mt, tt=tt,
                         max_rollout_moves=args.max_rollout_moves, want_rewards=False)
            wall = time.perf_counter() - t0
            kms = gpu.last_kernel_ms()
            o = r["out"]
            sims = int(o["iterations_run"].sum())
            print(json.dumps({"tool": "mcts_bench", "games": G, "iterations": it,
                              "max_rollout_moves": args.max_rollout_moves, "tt": not args.no_tt,
                              "simulations": sims, "rollouts": int(o["rollouts"].sum()),
                              "tt_hits": int(o["tt_hits"].sum()), "nodes_used_mean": float(o["nodes_used"].mean()),
                              "kernel_ms": kms, "wall_s": wall, "sims_per_s_kernel": sims / (kms * 1e-3),
                              "sims_per_s_wall": sims / wall, "status_nonzero": int((o["status"] != 0).sum())}),
                  flush=True)


if __name__ == "__main__":
    main()
