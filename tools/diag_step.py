"""Diagnostic: where does a bench step spend its time?  (GPU box only.)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from reinforcementlearning_blokus_amd import _native as N
from reinforcementlearning_blokus_amd.gpu import BlokusGPU, empty_state

gpu = BlokusGPU(0)
dev = torch.device("cuda", 0)
roots_np = gpu.advance(empty_state(), 256, 20, seed=5, root_index=np.zeros(256, dtype=np.int32))
roots = torch.from_numpy(roots_np.view(np.uint8).reshape(256, 256)).to(dev)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
idx = torch.arange(n, dtype=torch.int32, device=dev) % 256
out = torch.empty((n, 32), dtype=torch.uint8, device=dev)


def call(k):
    gpu.rollout(roots, n, semantics=N.SEM_ARENA, rng=N.RNG_PHILOX, seed=k, root_index=idx, out=out)


call(0)
torch.cuda.synchronize()
for k in range(5):
    t0 = time.perf_counter()
    call(k + 1)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    ms = gpu.last_kernel_ms()
    t3 = time.perf_counter()
    print(f"launch {1e3*(t1-t0):.3f} ms  sync {1e3*(t2-t1):.3f} ms  kernel(ev) {ms:.3f} ms  "
          f"last_kernel_ms call {1e3*(t3-t2):.3f} ms", flush=True)
# back-to-back without host syncs
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(5):
    ev[k][0].record()
    call(100 + k)
    ev[k][1].record()
torch.cuda.synchronize()
t1 = time.perf_counter()
print("5 back-to-back steps wall %.3f ms/step; torch events:" % (1e3 * (t1 - t0) / 5),
      [round(a.elapsed_time(b), 3) for a, b in ev], flush=True)
