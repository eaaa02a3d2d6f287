"""Config-3 playout rate when the boundary hands over HOST buffers (BK_MEM_HOST):
roots and root_index copied in, 32-B results copied back, every call synchronous.
DESIGN.md quotes this next to bench.py's device-resident rate (never as `value`)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reinforcementlearning_blokus_amd import _native as N  # noqa: E402
from reinforcementlearning_blokus_amd.gpu import BlokusGPU, empty_state  # noqa: E402

gpu = BlokusGPU(0)
games, rollouts = 256, 1024
roots = gpu.advance(empty_state(), games, 20, seed=20260301, root_index=np.zeros(games, np.int32))
n = games * rollouts
idx = (np.arange(n, dtype=np.int32) // rollouts).astype(np.int32)
for k in range(3):
    gpu.rollout(roots, n, semantics=N.SEM_ARENA, rng=N.RNG_PHILOX, seed=k, root_index=idx)
steps = 10
t0 = time.perf_counter()
for k in range(steps):
    res = gpu.rollout(roots, n, semantics=N.SEM_ARENA, rng=N.RNG_PHILOX, seed=100 + k, root_index=idx)
dt = (time.perf_counter() - t0) / steps
print(json.dumps({"mode": "host buffers (BK_MEM_HOST)", "playouts_per_call": n, "ms_per_call": dt * 1e3,
                  "sims_per_s": n / dt, "kernel_ms": gpu.last_kernel_ms()}))
