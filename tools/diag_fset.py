"""Diagnostic: frontier tables of k_rollout_fr (SEM_ADVANCE, k plies from the empty board)
against the host ABI's fset_place, ply by ply; prints the first disagreement."""
import sys

import numpy as np
import torch  # noqa: F401  (one HIP runtime: torch first)

from reinforcementlearning_blokus_amd import _native as N
from reinforcementlearning_blokus_amd.gpu import BlokusGPU, empty_state


def bits(plane):
    out = []
    for w in range(7):
        v = int(plane[w])
        while v:
            b = (v & -v).bit_length() - 1
            out.append(w * 64 + b)
            v &= v - 1
    return out


def main():
    gpu = BlokusGPU(0)
    seeds = np.array([[11, 12, 13, 14]], dtype=np.uint32)
    prev_s, prev_t = empty_state(), N.fset_new(1)
    for k in range(1, int(sys.argv[1]) if len(sys.argv) > 1 else 80):
        st, tb = gpu.rollout_frontier(empty_state(), N.fset_new(1), 1, semantics=N.SEM_ADVANCE, max_plies=k,
                                      compat_seeds=seeds)[:2]
        moved = [p for p in range(4) if not np.array_equal(st["planes"][0, p], prev_s["planes"][0, p])]
        host = prev_t.copy()
        if moved:
            p = moved[0]
            new = sorted(set(bits(st["planes"][0, p])) - set(bits(prev_s["planes"][0, p])))
            N.fset_place(host, st[:1], p, new)
            if host.tobytes() != tb.tobytes():
                print("ply", k, "player", p, "cells", new)
                for q in range(4):
                    print(" q", q, "gpu ", N.fset_list(tb, q))
                    print("      host", N.fset_list(host, q))
                    print("      before", N.fset_list(prev_t, q))
                return 1
        prev_s, prev_t = st, tb
    print("tables agree for", k, "plies")
    return 0


if __name__ == "__main__":
    sys.exit(main())
