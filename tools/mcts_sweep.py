"""Tree-phase batch threshold sweep (BK_TREE_BATCH) for bk_mcts: wall time of full
searches per threshold, results checked identical across thresholds."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from reinforcementlearning_blokus_amd import _native as N  # noqa: E402
from reinforcementlearning_blokus_amd.gpu import BlokusGPU  # noqa: E402
from reinforcementlearning_blokus_amd.workloads import MctsBatch, frontier_roots  # noqa: E402


def main():
    gpu = BlokusGPU(0)
    cases = [(65536, int(os.environ.get("SWEEP_ITERS", "1024")), N.MCTS_ROLLOUT_RANDOM),
             (4096, 64, N.MCTS_ROLLOUT_HEURISTIC)]
    for games, iters, pol in cases:
        roots, sets = frontier_roots(gpu, games, 20, seed=11)
        b = MctsBatch(gpu, roots, sets, iterations=iters, seed0=3)
        ref = None
        for tb in [int(x) for x in os.environ.get("SWEEP_TB", "1,4,8,12,16,24,32").split(",")]:
            os.environ["BK_TREE_BATCH"] = str(tb)
            b.reset()
            t = time.perf_counter()
            b.gpu.mcts_device(b.roots, b.sets, b.players, b.root_hash, b.zobrist, b.zidx, b.mt, b.log_table, b.nodes,
                              b.out, iterations=iters, tt_keys=b.tt_keys, tt_vals=b.tt_vals, tt_count=b.tt_count,
                              rollout_policy=pol)
            gpu.synchronize()
            dt = time.perf_counter() - t
            r = b.results()
            key = np.stack([r["best_move"], r["rollouts"], r["tt_hits"], r["nodes_used"]]).astype(np.int64)
            same = ref is None or bool((key == ref).all())
            ref = key if ref is None else ref
            print(json.dumps({"games": games, "iters": iters, "policy": int(pol), "tree_batch": tb,
                              "s": round(dt, 3), "sims_per_s": round(games * iters / dt), "identical": same,
                              "status_or": int(np.bitwise_or.reduce(r["status"]))}), flush=True)


if __name__ == "__main__":
    main()
