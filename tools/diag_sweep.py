"""Diagnostic sweep (GPU box only): rollout kernel time vs residency and batch size."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from reinforcementlearning_blokus_amd import _native as N
from reinforcementlearning_blokus_amd.gpu import BlokusGPU, empty_state

dev = torch.device("cuda", 0)
base = BlokusGPU(0)
roots_np = base.advance(empty_state(), 256, 20, seed=5, root_index=np.zeros(256, dtype=np.int32))
roots = torch.from_numpy(roots_np.view(np.uint8).reshape(256, 256)).to(dev)
for bpc in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,2,3").split(",")]:
    os.environ["BK_BLOCKS_PER_CU"] = str(bpc)
    gpu = BlokusGPU(0)
    for n in (262144, 1048576):
        idx = torch.arange(n, dtype=torch.int32, device=dev) // (n // 256)
        out = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        gpu.rollout(roots, n, seed=1, root_index=idx, out=out)
        torch.cuda.synchronize()
        ms = []
        for k in range(3):
            gpu.rollout(roots, n, seed=2 + k, root_index=idx, out=out)
            torch.cuda.synchronize()
            ms.append(gpu.last_kernel_ms())
        m = min(ms)
        print(f"bpc={bpc} n={n}: kernel {m:.3f} ms -> {n / m * 1e3 / 1e6:.2f} M sims/s", flush=True)
