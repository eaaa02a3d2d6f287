"""Profiling target (GPU box only): warm up, then exactly one timed k_rollout launch of the
bench workload (config 3, 262,144 playouts) so per-dispatch counters map to one launch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from reinforcementlearning_blokus_amd import _native as N
from reinforcementlearning_blokus_amd.gpu import BlokusGPU, empty_state

n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
dev = torch.device("cuda", 0)
gpu = BlokusGPU(0)
roots_np = gpu.advance(empty_state(), 256, 20, seed=20260301, root_index=np.zeros(256, dtype=np.int32))
roots = torch.from_numpy(roots_np.view(np.uint8).reshape(256, 256)).to(dev)
idx = torch.arange(n, dtype=torch.int32, device=dev) // (n // 256)
out = torch.empty((n, 32), dtype=torch.uint8, device=dev)
for k in range(2):
    gpu.rollout(roots, n, seed=k, root_index=idx, out=out)
torch.cuda.synchronize()
print("done", gpu.last_kernel_ms())
