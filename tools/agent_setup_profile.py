"""cProfile of the config-4 agent setup (_device_agents, 1,024 games) inside a process set
up as bench.py's config-4 rank is (torch on the GPU, host cores pinned).  Diagnostic."""
import cProfile
import io
import pstats
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch  # noqa: E402

import bench  # noqa: E402
from reinforcementlearning_blokus_amd.arena import runner as R  # noqa: E402
from reinforcementlearning_blokus_amd.arena.config import RunConfig  # noqa: E402

torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
pinned = "--pin" in sys.argv
if pinned:
    print(bench.pin_host_cores(None))
cfg = RunConfig.from_dict({"agents": bench.CONFIG4_AGENTS, "num_games": 1024, "seed": 20260301,
                           "seat_policy": "round_robin"})
idx = list(range(1024))
seats = [R.seat_assignment_for_game(cfg.agent_names, gi, R.game_seed_from_run_seed(cfg.seed, gi), cfg.seat_policy)
         for gi in idx]
for rep in range(3):
    t = time.perf_counter()
    R._device_agents(cfg, seats, idx)
    print("pinned" if pinned else "unpinned", rep, time.perf_counter() - t)
pr = cProfile.Profile()
pr.enable()
R._device_agents(cfg, seats, idx)
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(14)
print(s.getvalue()[:3000])
