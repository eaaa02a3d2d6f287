import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
from reinforcementlearning_blokus_amd import _native as N
from reinforcementlearning_blokus_amd.gpu import BlokusGPU
from tests.helpers import POS, fset_of, pack_many, replay
gpu = BlokusGPU(0)
recs = [{"position": i} for i in range(8, 56)]
boards = [replay(POS[r["position"]]) for r in recs]
sets = np.array([fset_of(POS[r["position"]]) for r in recs], dtype=N.FSET_DTYPE)
roots = pack_many(boards)
for n in (512, 1024, 4096):
    idx = (np.arange(n) % len(recs)).astype(np.int32)
    seeds = (np.arange(4 * n, dtype=np.uint64).reshape(n, 4) * 40503 % 2**31).astype(np.uint32)
    outs = {}
    for t in (0, 24, 0, 24, 64):
        gpu.tune(MERGE=t)
        r = gpu.rollout_frontier(roots, sets, n, compat_seeds=seeds, root_index=idx)
        if t in outs:
            print(n, t, "repeat equal", np.array_equal(outs[t], r), flush=True)
        else:
            outs[t] = r
    for t in (24, 64):
        bad = np.nonzero(outs[t] != outs[0])[0]
        print(n, t, "differ", len(bad), bad[:20].tolist(), flush=True)
        for i in bad[:4]:
            print("   ", i, outs[0][i], outs[t][i], flush=True)
    # philox
    outs = {}
    for t in (0, 24):
        gpu.tune(MERGE=t)
        outs[t] = gpu.rollout_frontier(roots, sets, n, rng=N.RNG_PHILOX, seed=3, root_index=idx)
    bad = np.nonzero(outs[24] != outs[0])[0]
    print(n, "philox differ", len(bad), bad[:20].tolist(), flush=True)
    outs = {}
    for t in (0, 24):
        gpu.tune(MERGE=t)
        outs[t] = gpu.rollout(roots, n, rng=N.RNG_NUMPY_MT, compat_seeds=seeds, root_index=idx)
    bad = np.nonzero(outs[24] != outs[0])[0]
    print(n, "naive compat differ", len(bad), bad[:20].tolist(), flush=True)
