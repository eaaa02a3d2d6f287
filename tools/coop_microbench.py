#!/usr/bin/env python3
"""Kernel time of the cooperative MCTS kernels alone (diagnostic A/B, GPU box): 512
searches x 64 iterations from 24-ply roots with HeuristicAgent rollouts (k_mcts_coop_h,
a config-4 arena round) and with RandomAgent rollouts (k_mcts_coop), `--reps` launches
each; prints one JSON line per kernel with the launch times (HIP events).  The library is
the in-tree one or BK_LIB_PATH's."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 5
    from reinforcementlearning_blokus_amd import _native as N
    from reinforcementlearning_blokus_amd.gpu import BlokusGPU
    from reinforcementlearning_blokus_amd.workloads import MctsBatch, frontier_roots
    gpu = BlokusGPU(0)
    gpu.tune(MCTS_COOP=1)
    roots, sets = frontier_roots(gpu, 512, 24, seed=11)
    for policy in (N.MCTS_ROLLOUT_HEURISTIC, N.MCTS_ROLLOUT_RANDOM):
        b = MctsBatch(gpu, roots, sets, iterations=64, seed0=3)
        ms = []
        for _ in range(reps + 1):
            b.reset()
            b.run(rollout_policy=policy, on_chunk=lambda k: ms.append(gpu.last_kernel_ms()))
        ms = ms[1:]
        print(json.dumps({"kernel": gpu.last_kernel(), "searches": 512, "iterations": 64, "ms": ms,
                          "ms_min": min(ms), "ms_mean": sum(ms) / len(ms)}), flush=True)
        if "--state-rows" in sys.argv:  # the same searches through BK_MCTS_STATE_ROWS (agent rows = searches)
            import torch
            n = 512
            zob = b.zobrist[b.zidx.long()].contiguous()  # one zobrist row per search: zidx = g
            zi = torch.arange(n, dtype=torch.int32, device=zob.device)
            ms = []
            hb = None
            if "--done" in sys.argv:  # with per-search result words into mapped host memory
                hb = N.HostBuffer(8 * n, np.uint64)
                b.gpu.handle.set_done(hb.ptr)
            for _ in range(reps + 1):
                b.reset()
                if hb is not None:
                    hb.array[:] = 0
                b.gpu.mcts_device(b.roots, b.sets, b.players, b.root_hash, zob, zi, b.mt, b.log_table, b.nodes, b.out,
                                  iterations=64, tt_keys=b.tt_keys, tt_vals=b.tt_vals, tt_count=b.tt_count,
                                  max_rollout_moves=b.max_rollout_moves, rollout_policy=policy, state_rows=True)
                ms.append(gpu.last_kernel_ms())
            ms = ms[1:]
            tag = "+state_rows" + ("+done" if hb is not None else "")
            if hb is not None:
                b.gpu.handle.set_done(None)
                tag += f" ({int(np.count_nonzero(hb.array >> np.uint64(63)))} words)"
            print(json.dumps({"kernel": gpu.last_kernel() + tag, "searches": n, "ms": ms,
                              "ms_min": min(ms), "ms_mean": sum(ms) / len(ms)}), flush=True)


if __name__ == "__main__":
    main()
