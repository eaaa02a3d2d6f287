"""Config 4 on one GPU: an all-random arena run of N games (reference seeding, frontier
order, per-seat numpy streams) played by run_games_gpu; prints games/s.
usage: python tools/arena_bench.py [num_games]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reinforcementlearning_blokus_amd.arena import RunConfig, run_games_gpu  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
cfg = RunConfig.from_dict({"agents": [{"name": f"r{i}", "type": "random"} for i in range(4)], "num_games": n,
                           "seed": 20260301, "seat_policy": "randomized"})
run_games_gpu(cfg, range(64))  # warm-up
t0 = time.perf_counter()
recs = run_games_gpu(cfg, range(n))
dt = time.perf_counter() - t0
print(json.dumps({"workload": "config4 all-random arena (frontier order, reference seeds)", "games": n,
                  "seconds": dt, "games_per_s": n / dt,
                  "mean_moves": sum(r["moves_made"] for r in recs) / n}))
