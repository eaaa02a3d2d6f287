#!/usr/bin/env python3
"""Where does a playout / search ply spend its time?  (GPU box; diagnostic only.)

Builds (on the CPU side, beforehand: `python tools/sections.py --build`) a second copy
of the HIP library with -DBK_SECTION_PROF into tools/_prof/, then (on the box) loads it
through BK_LIB_PATH, runs k_rollout (naive order), k_rollout_fr (frontier order) and
k_mcts on config-3-like inputs, and prints each section's share of the per-wave
shader-clock cycles (bk_debug_sections)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get("BK_SECTIONS_LIB") or os.path.join(ROOT, "tools", "_prof", "libblokus_hip_sections.so")

NAMES = {0: "loop tail", 1: "game start/finish", 2: "derive+movegen counts", 3: "draw+pick+rows->LDS",
         4: "locate", 5: "apply", 6: "frontier place", 8: "mcts: tree select/replay/backprop/start",
         9: "mcts: derive+movegen", 10: "mcts: expand bookkeeping/draw+pick", 11: "mcts: locate_frontier",
         12: "mcts: expand place/copies/TT", 13: "mcts: loop tail", 14: "mcts: rollout place",
         15: "(resizes, inside the set ops: not a section)"}


# k_rollout_fr's frontier place, split (the place_frontier marks)
FR_NAMES = {7: "frontier ops windows", 8: "place: stage load + LDS write", 9: "place: set ops",
            6: "place: write-back"}


def build():
    sys.path.insert(0, ROOT)
    from reinforcementlearning_blokus_amd import build as B
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    B.compile_library(LIB, defines=("BK_SECTION_PROF",))
    print(LIB)


def run():
    os.environ["BK_LIB_PATH"] = LIB
    sys.path.insert(0, ROOT)
    import ctypes as C

    import numpy as np
    from reinforcementlearning_blokus_amd import _native as N
    from reinforcementlearning_blokus_amd.gpu import BlokusGPU, MctsTT, empty_state
    from reinforcementlearning_blokus_amd.mcts.zobrist import ZobristHash, flat_keys, hash_states
    gpu = BlokusGPU(0)
    L = N.load()
    buf = (C.c_uint64 * 16)()

    def read(tag, extra, names=None):
        rc = L.bk_debug_sections(gpu.handle._h, buf, 16, 1)
        assert rc == 0, rc
        tot = sum(buf)
        nm = {**NAMES, **(names or {})}
        rows = {nm.get(i, str(i)): round(buf[i] / tot, 4) for i in range(16) if buf[i]}
        print(json.dumps({"run": tag, **extra, "cycles": tot, "share": rows, "raw": list(buf)}), flush=True)

    L.bk_debug_sections(gpu.handle._h, buf, 16, 1)
    G, R = 256, 1024
    roots = gpu.advance(empty_state(), G, 20, seed=5, root_index=np.zeros(G, dtype=np.int32))
    idx = np.repeat(np.arange(G, dtype=np.int32), R)
    gpu.rollout(roots, G * R, semantics=N.SEM_ARENA, rng=N.RNG_PHILOX, seed=1, root_index=idx)
    read("k_rollout naive", {"kernel_ms": gpu.last_kernel_ms()})
    froots, fsets = gpu.rollout_frontier(empty_state(), N.fset_new(1), G, semantics=N.SEM_ADVANCE,
                                         rng=N.RNG_PHILOX, seed=5, max_plies=20,
                                         root_index=np.zeros(G, dtype=np.int32))
    gpu.rollout_frontier(froots, fsets, G * R, semantics=N.SEM_ARENA, rng=N.RNG_PHILOX, seed=1, root_index=idx)
    read("k_rollout_fr", {"kernel_ms": gpu.last_kernel_ms()}, FR_NAMES)
    for games in (4096, 65536):
        froots, fsets = gpu.rollout_frontier(empty_state(), N.fset_new(1), games, semantics=N.SEM_ADVANCE,
                                             rng=N.RNG_PHILOX, seed=5, max_plies=20,
                                             root_index=np.zeros(games, dtype=np.int32))
        keys = flat_keys(ZobristHash(seed=3))
        mt = np.zeros((games, 625), np.uint32)
        for g in range(games):
            st = np.random.RandomState(g).get_state()
            mt[g, :624], mt[g, 624] = st[1], st[2]
        gpu.mcts(froots, fsets, froots["current_player"].copy(), hash_states(froots, keys), iterations=16,
                 zobrist=keys[None], mt_state=mt, tt=MctsTT(games, cap=64), want_rewards=False)
        read("k_mcts", {"games": games, "iterations": 16, "kernel_ms": gpu.last_kernel_ms()})


def run_mcts():
    """k_mcts sections in the config-5 regime (65,536 searches, deep trees: a warm-up of
    `iterations` then a measured chunk of 64 more) and k_mcts_h (heuristic rollouts)."""
    os.environ["BK_LIB_PATH"] = LIB
    sys.path.insert(0, ROOT)
    import ctypes as C

    from reinforcementlearning_blokus_amd import _native as N
    from reinforcementlearning_blokus_amd.gpu import BlokusGPU
    from reinforcementlearning_blokus_amd.workloads import MctsBatch, frontier_roots
    gpu = BlokusGPU(0)
    L = N.load()
    buf = (C.c_uint64 * 16)()

    def read(tag, extra, names=None):
        rc = L.bk_debug_sections(gpu.handle._h, buf, 16, 1)
        assert rc == 0, rc
        tot = sum(buf)
        nm = {**NAMES, **(names or {})}
        rows = {nm.get(i, str(i)): round(buf[i] / tot, 4) for i in range(16) if buf[i]}
        print(json.dumps({"run": tag, **extra, "cycles": tot, "share": rows, "raw": list(buf)}), flush=True)

    runs = ((65536, int(os.environ.get("BK_SECT_ITERS", "512")), N.MCTS_ROLLOUT_RANDOM),
            (4096, 96, N.MCTS_ROLLOUT_HEURISTIC))
    if os.environ.get("BK_SECT_ITERS"):
        runs = runs[:1]
    for games, iters, policy in runs:
        roots, sets = frontier_roots(gpu, games, 20, seed=11)
        b = MctsBatch(gpu, roots, sets, iterations=iters, seed0=3)
        gpu.mcts_device(b.roots, b.sets, b.players, b.root_hash, b.zobrist, b.zidx, b.mt, b.log_table, b.nodes,
                        b.out, iterations=iters, tt_keys=b.tt_keys, tt_vals=b.tt_vals, tt_count=b.tt_count,
                        chunk=64, stop_after=iters - 64, rollout_policy=policy)
        L.bk_debug_sections(gpu.handle._h, buf, 16, 1)
        gpu.mcts_device(b.roots, b.sets, b.players, b.root_hash, b.zobrist, b.zidx, b.mt, b.log_table, b.nodes,
                        b.out, iterations=iters, tt_keys=b.tt_keys, tt_vals=b.tt_vals, tt_count=b.tt_count,
                        chunk=64, resume_from=iters - 64, rollout_policy=policy)
        # k_mcts splits its tree phase: 0 select, 1 replay, 2 game start/finish/complete;
        # and its place: 3 frontier ops windows, 4 slab rows, 5 set ops (k_mcts_pair's stage)
        NAMES.update({0: "mcts tree: select", 1: "mcts tree: replay", 2: "mcts tree: start/finish/terminal",
                      3: "mcts place: ops windows", 4: "mcts place: piece cells + slab rows",
                      5: "mcts place: set ops", 14: "mcts place: write-back + rollout tail"})
        read("k_mcts" if policy == N.MCTS_ROLLOUT_RANDOM else "k_mcts_h",
             {"games": games, "iterations": f"{iters - 64}..{iters}", "kernel_ms": gpu.last_kernel_ms()})


def run_coop():
    """k_mcts_coop(_h) sections (one wave per search): 512 searches x 64 iterations with
    heuristic rollouts (a config-4 arena round) and with random rollouts."""
    os.environ["BK_LIB_PATH"] = LIB
    os.environ["BK_MCTS_COOP"] = "1"
    sys.path.insert(0, ROOT)
    import ctypes as C

    from reinforcementlearning_blokus_amd import _native as N
    from reinforcementlearning_blokus_amd.gpu import BlokusGPU
    from reinforcementlearning_blokus_amd.workloads import MctsBatch, frontier_roots
    gpu = BlokusGPU(0)
    L = N.load()
    buf = (C.c_uint64 * 16)()
    names = {0: "tree", 1: "derive+rows", 2: "lane orientations+scan", 3: "draw+pick (rest)",
             4: "locate / heuristic walk", 5: "expansion / rollout tail", 6: "heuristic: list moves",
             7: "heuristic: e pass + scan", 8: "piece cells + frontier ops windows", 9: "place: slab rows",
             10: "place: set ops", 11: "place: write-back / copy"}
    for policy in (N.MCTS_ROLLOUT_HEURISTIC, N.MCTS_ROLLOUT_RANDOM):
        roots, sets = frontier_roots(gpu, 512, 24, seed=11)
        b = MctsBatch(gpu, roots, sets, iterations=64, seed0=3)
        L.bk_debug_sections(gpu.handle._h, buf, 16, 1)
        b.run(rollout_policy=policy)
        rc = L.bk_debug_sections(gpu.handle._h, buf, 16, 1)
        assert rc == 0, rc
        tot = sum(buf)
        rows = {names.get(i, str(i)): round(buf[i] / tot, 4) for i in range(16) if buf[i]}
        print(json.dumps({"run": "k_mcts_coop_h" if policy == N.MCTS_ROLLOUT_HEURISTIC else "k_mcts_coop",
                          "searches": 512, "iterations": 64, "kernel_ms": gpu.last_kernel_ms(), "cycles": tot,
                          "share": rows}), flush=True)


if __name__ == "__main__":
    if "--build" in sys.argv:
        build()
    elif "--coop" in sys.argv:
        run_coop()
    elif "--mcts" in sys.argv:
        run_mcts()
    else:
        run()
