#!/usr/bin/env python3
"""Where do k_movegen_m's extra written bytes come from?  (GPU box; diagnostic only.)

Config-2 inputs (4,096 boards, plies 16..40, player to move), then bk_movegen_mask on
device buffers in three modes, 20 launches each, in this order: masks + counts (the
bench's call), masks only (out_count NULL: no count atomics), counts only.  Run under
rocprofv3 --pmc WRITE_SIZE (or FETCH_SIZE) and compare the launches of each mode."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from reinforcementlearning_blokus_amd import _native as N
    from reinforcementlearning_blokus_amd.gpu import BlokusGPU, empty_state
    gpu = BlokusGPU(0)
    rng = np.random.RandomState(7)
    plies = rng.randint(16, 41, size=4096)
    parts = []
    for m in range(16, 41):
        k = int((plies == m).sum())
        if k:
            parts.append(gpu.advance(empty_state(), k, m, seed=7 * 41 + m, root_index=np.zeros(k, dtype=np.int32)))
    st = np.concatenate(parts)
    n = len(st)
    dev = torch.device("cuda", 0)
    states = torch.from_numpy(st.view(np.uint8).reshape(n, 256).copy()).to(dev)
    players = torch.from_numpy((st["current_player"] & 3).astype(np.uint8)).to(dev)
    cnt = torch.zeros(n, dtype=torch.int32, device=dev)
    masks = torch.zeros((n, N.N_ORIENTS, 7), dtype=torch.int64, device=dev)
    gpu._stream_from_torch()
    for mode, (mp, cp) in (("masks+counts", (masks.data_ptr(), cnt.data_ptr())), ("masks", (masks.data_ptr(), 0)),
                           ("counts", (0, cnt.data_ptr()))):
        for _ in range(20):
            gpu.handle.movegen_mask(states.data_ptr(), players.data_ptr(), n, mp, cp, N.MEM_DEVICE)
        torch.cuda.synchronize()
        print(mode, "done", flush=True)


if __name__ == "__main__":
    main()
