"""Which start order of the two HIP runtimes in one process (torch's bundled one and
/opt/rocm's, linked by libblokus_hip.so) leaves both able to use the GPU.
  python tools/runtime_order_probe.py ours|torch"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reinforcementlearning_blokus_amd import _native as N  # noqa: E402

order = sys.argv[1]
if order == "ours":
    # bypass _native.load()'s torch-first import: ctypes-load the library on its own
    import ctypes
    L = ctypes.CDLL(N.LIB_PATH)
    h = ctypes.c_void_p()
    assert L.bk_create(0, 0, ctypes.byref(h)) == 0
    print("ours ok", flush=True)
    import torch
    print("torch avail", torch.cuda.is_available(), flush=True)
    x = torch.ones(4, device="cuda")
    print("torch ok", float(x.sum()), flush=True)
else:
    import torch
    print("torch avail", torch.cuda.is_available(), flush=True)
    x = torch.ones(4, device="cuda")
    print("torch ok", float(x.sum()), flush=True)
    h = N.Handle(0)
    print("ours ok", flush=True)
# Measured on the MI355X box (round 1): "torch" order -> both work; "ours" order -> torch
# reports "No HIP GPUs are available" (two runtimes).  Hence _native.load() imports torch
# before it loads the library, so the process has one HIP runtime.
