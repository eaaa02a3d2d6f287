"""Build the in-tree HIP library (gfx950) and the CPU oracle (test infrastructure)."""
from __future__ import annotations

import os
import shutil
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(_HERE)
SRC = os.path.join(_HERE, "csrc", "blokus_kernels.hip")
OUT = os.path.join(_HERE, "_lib", "libblokus_hip.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def build_native(force: bool = False, verbose: bool = False) -> str:
    deps = [SRC, os.path.join(_HERE, "csrc", "orient_table.h"), os.path.join(ROOT, "include", "blokus_hip.h")]
    if not force and os.path.exists(OUT) and all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in deps):
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC",
           "-Wno-unused-command-line-argument", "-o", OUT + ".tmp", SRC]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


def build_oracle() -> None:
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


if __name__ == "__main__":
    print(build_native(force=True, verbose=True))
    build_oracle()
