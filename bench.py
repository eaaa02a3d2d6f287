#!/usr/bin/env python3
"""Headline benchmark: MCTS random-rollout simulations/sec (20x20, 4 players).

One "step" = one batch of the config-3 workload (BASELINE.json configs[2]):
256 concurrent self-play games, 1,024 random rollouts per game-move, i.e. 262,144
terminal random playouts (arena semantics: pass when stuck, game over when nobody
can move, GameResult scoring) from 256 synthetic mid-game positions (20 random
plies from the empty board), all resident in HBM before the timed region.

N>1: one process per GPU (torchrun), each rank plays its own 256 games (weak
scaling, no data-path collective); after the timed region the per-rank result
checksums are all-gathered over RCCL.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "MCTS random-rollout simulations/sec (20x20, 4p) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
# VALU int32 peak: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz.  Measured (tools/valu_probe2.hip):
# v_or/v_xor/v_lshrrev/v_add/v_bitop3 issue in ~2.5 cycles per wave64 with >= 2 waves per
# SIMD (32 lanes/clk); v_lshl_or/v_lshlrev/v_bcnt/v_or3 take ~4.3-4.6 (half rate)
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
# Single-issue rate (one wave64 VALU op per 4 cycles per SIMD): what any stream holding
# slow ops (v_bcnt, SGPR operands, left shifts ...) gets -- k_rollout's case
VALU_SINGLE_TOPS = 256 * 4 * 16 * 2.4e9 / 1e12


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--games", type=int, default=256)
    ap.add_argument("--rollouts", type=int, default=1024)
    ap.add_argument("--root-plies", type=int, default=20)
    ap.add_argument("--seed", type=int, default=20260301)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--order", choices=("naive", "frontier"), default="naive",
                    help="in-kernel move order: naive (default) or the reference's frontier order "
                         "(CPython set tables carried per game)")
    return ap.parse_args()


def cpu_baseline(roots_np, seconds: float):
    """Oracle (C restatement, reference frontier algorithm + game-over check after every
    move) timed on this host's cores on a bounded sample of the same workload."""
    from oracle import pyoracle as O
    threads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))
    st = (O.State * len(roots_np)).from_buffer_copy(roots_np.tobytes())
    n = 16 * threads
    t0 = time.perf_counter()
    O.batch_playouts(st, n, 1, threads=threads)
    dt = time.perf_counter() - t0
    # scale the sample to ~`seconds` of wall time
    n2 = max(n, int(n * seconds / max(dt, 1e-3)))
    t0 = time.perf_counter()
    O.batch_playouts(st, n2, 2, threads=threads)
    dt = time.perf_counter() - t0
    return {"value": n2 / dt, "unit": "sims/s", "cores": threads, "kind": "port",
            "sample": f"{n2} arena playouts from the same {len(roots_np)} roots, "
                      f"oracle/blokus_oracle.c (reference frontier movegen order), {threads} threads, {dt:.1f} s"}


def main():
    args = parse()
    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from reinforcementlearning_blokus_amd import _native as N
    from reinforcementlearning_blokus_amd.gpu import BlokusGPU, empty_state

    gpu = BlokusGPU(local)
    dev = torch.device("cuda", local)
    seed = args.seed + 1_000_003 * rank
    # synthetic mid-game roots, generated on the GPU (BK_SEM_ADVANCE from the empty board)
    if args.order == "frontier":
        roots_np, sets_np = gpu.rollout_frontier(empty_state(), N.fset_new(1), args.games,
                                                 semantics=N.SEM_ADVANCE, rng=N.RNG_PHILOX, seed=seed,
                                                 max_plies=args.root_plies,
                                                 root_index=np.zeros(args.games, dtype=np.int32))
        sets = torch.from_numpy(sets_np.view(np.uint8).reshape(args.games, -1).copy()).to(dev)
    else:
        roots_np = gpu.advance(empty_state(), args.games, args.root_plies, seed=seed,
                               root_index=np.zeros(args.games, dtype=np.int32))
    roots = torch.from_numpy(roots_np.view(np.uint8).reshape(args.games, 256)).to(dev)
    n = args.games * args.rollouts
    # game j's rollouts are contiguous (one wave plays 64 rollouts of the same game)
    idx = torch.arange(n, dtype=torch.int32, device=dev) // args.rollouts
    out = torch.empty((n, 32), dtype=torch.uint8, device=dev)

    stream = torch.cuda.Stream(dev)  # our kernels and the timing events share this stream
    plies_acc = torch.zeros(1, dtype=torch.int64, device=dev)

    def step(k):
        if args.order == "frontier":
            gpu.rollout_frontier(roots, sets, n, semantics=N.SEM_ARENA, rng=N.RNG_PHILOX, seed=seed * 7919 + k,
                                 root_index=idx, out=out)
            return
        gpu.rollout(roots, n, semantics=N.SEM_ARENA, rng=N.RNG_PHILOX, seed=seed * 7919 + k, root_index=idx,
                    out=out)

    def count_plies():
        plies_acc.add_(out[:, 10:12].contiguous().view(torch.int16).to(torch.int64).sum())

    with torch.cuda.stream(stream):
        for k in range(args.warmup):
            step(k)
            count_plies()
        plies_acc.zero_()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.steps)]
        t0 = time.perf_counter()
        for k in range(args.steps):
            events[k][0].record(stream)
            step(1000 + k)
            events[k][1].record(stream)
            count_plies()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
    kernel_ms = [a.elapsed_time(b) for a, b in events]
    plies = int(plies_acc.item())
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    tot = torch.tensor([n * args.steps, plies], dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        # RCCL gather of the last step's terminal results (32 B per playout) over xGMI,
        # outside the timed region; rank r's playouts are global games r (mod W)
        from reinforcementlearning_blokus_amd.shard import gather_results
        gather_results(out, n * world, rank, world, dist)
    elapsed = float(t.item())
    sims, all_plies = float(tot[0].item()), float(tot[1].item())
    value = sims / elapsed

    if rank == 0:
        avg_ms = sum(kernel_ms) / len(kernel_ms)
        plies_per_sim = all_plies / sims
        # SURVEY 8(d) algorithmic bytes: 256 B state read + 256 B write per ply, 32 B result
        bytes_per_sim = 512.0 * plies_per_sim + 32.0
        achieved = (n * bytes_per_sim) / (avg_ms * 1e-3) / 1e9
        traffic = valu_insts = None
        tpath = os.path.join(ROOT, "profiles", "traffic_latest.json")
        if os.path.exists(tpath) and args.order == "naive":  # PMC pass is of k_rollout
            try:
                tj = json.load(open(tpath))
                traffic, valu_insts = tj.get("bytes_per_launch"), tj.get("valu_insts_per_launch")
            except (OSError, ValueError):
                traffic = valu_insts = None
        # VALU view (the real limiter): wave64 VALU instructions per launch
        # from the committed PMC pass (SQ_INSTS_VALU, same workload) x 64 lanes over the
        # live launch time, against the dual-issue int32 VALU peak of 32 lanes/clk/SIMD
        valu_tops = valu_insts * 64 / (avg_ms * 1e-3) / 1e12 if valu_insts else None
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "sims/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic",
            "config": {"workload": "config3: 256 concurrent games x 1024 random rollouts (arena semantics, "
                                   f"{args.order} move order, Philox RNG) from GPU-generated 20-ply positions",
                       "games": args.games, "rollouts_per_game": args.rollouts, "root_plies": args.root_plies,
                       "playouts_per_step": n, "parallelism": f"dp{world} (independent games per rank)"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "k_rollout_fr" if args.order == "frontier" else "k_rollout",
                         "kernel_ms": avg_ms, "plies_per_sim": plies_per_sim},
            "compute_roofline": {"bound": "valu_int32", "achieved": valu_tops, "peak": VALU_PEAK_TOPS,
                                 "unit": "Tlane-op/s", "frac": valu_tops / VALU_PEAK_TOPS if valu_tops else None,
                                 "peak_single_issue": VALU_SINGLE_TOPS,
                                 "frac_single_issue": valu_tops / VALU_SINGLE_TOPS if valu_tops else None,
                                 "valu_insts_per_launch": valu_insts},
        }
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(roots_np, args.cpu_seconds)
            line["cpu_baseline"]["gpu_over_cpu"] = value / line["cpu_baseline"]["value"]
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
