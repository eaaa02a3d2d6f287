#!/usr/bin/env python3
"""Headline benchmark: MCTS random-rollout simulations/sec (20x20, 4 players).

Default workload (`--workload config3`, BASELINE.json configs[2]) -- one "step" = 256
concurrent self-play games x 1,024 random rollouts per game-move = 262,144 terminal
random playouts (arena semantics: pass when stuck, game over when nobody can move,
GameResult scoring) from 256 synthetic mid-game positions (20 random plies from the
empty board), all resident in HBM before the timed region.  The line's `value` is the
reference as shipped: its default frontier move order (BLOKUS_USE_FRONTIER_MOVEGEN=1,
engine/move_generator.py:66, :148; kernel k_rollout_fr).  The default line also carries:
  naive_order  the same measurement in naive order (BLOKUS_USE_FRONTIER_MOVEGEN=0, k_rollout)
  config5      BASELINE configs[4]: 65,536 MCTSAgent searches x 4,096 iterations (one
               launch after a 64-iteration warmup), strong scaling over the ranks
  config4      BASELINE configs[3]: 1,024 arena games per rank (8,192 at 8 GPUs) after one
               warm-up batch
each with its own value, ms_per_step, roofline and (one GPU) cpu_baseline.

Other workloads (one JSON line each, same contract):
  --workload config5  BASELINE.json configs[4]: 65,536 concurrent MCTSAgent searches x
                      4,096 iterations (UCT + Zobrist TT in HBM + 50-ply RandomAgent
                      rollouts, reference frontier move order, bit-exact); one step =
                      the whole batch of searches.  N>1: the 65,536 games are sharded
                      over the ranks (strong scaling).
  --workload config2  BASELINE.json configs[1]: batched legal-move generation for 4,096
                      synthetic mid-game boards (plies 16..40), player to move (and
                      --all-players: all 4); one step = one bk_movegen_mask launch.

N>1: one process per GPU, weak scaling for config3 (each rank plays its own 256 games,
no data-path collective); after the timed region the per-rank results are all-gathered
over RCCL.  Prints ONE JSON line on rank 0.  Either launch works:
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
  python bench.py --gpus N        (bench.py starts the N rank processes itself)
`--gpus` must equal the process group's size; `n_gpus` is taken from the group.
`--selftest [--gpus N]` checks the N-rank launch/shard/gather path on CPU with gloo.
"""
from __future__ import annotations

import argparse
import json
import math
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
# Reference engine (Python) rates measured in the build container (SURVEY.md 6,
# BASELINE.md): it cannot run on the GPU box, so these are carried, not re-timed.
REF_PY_ARENA_SIMS_PER_CORE = 5.5      # terminal random playout from ply 20
REF_PY_MCTS_RANDOM_SIMS = 8.6         # MCTSAgent + RandomAgent rollouts, 100 iterations
REF_PY_MOVEGEN_BOARDS_PER_CORE = 162  # get_legal_moves at ply 20
REF_CONTAINER = "8-vCPU Intel Xeon build container, Python 3.10.12, numpy 2.2.6"
# SURVEY 8(d) algorithmic bytes
STATE_B, RESULT_B = 256, 32
MOVEGEN_B = 256 + 5096  # state in + dense 91 x 400-bit mask out, per board-player


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one process per GPU).  Under torch.distributed.run it must equal WORLD_SIZE; "
                         "run directly with N > 1, bench.py starts the N rank processes itself")
    ap.add_argument("--selftest", action="store_true",
                    help="CPU check of the N-rank path (gloo): launch, shard, gather, compare with one process")
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default: 20; config5: 1)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default: 3; config5: 1, "
                                                              "a 64-iteration chunk)")
    ap.add_argument("--share-device", action="store_true",
                    help="rehearsal of the N-rank path on a one-GPU box: every rank runs on cuda:0 and the "
                         "process group is gloo (tests only; never a scaling number)")
    ap.add_argument("--check-gather", action="store_true",
                    help="config3, N ranks: rank 0 checks the gathered records against one launch of the "
                         "whole job's games")
    ap.add_argument("--workload", choices=("config3", "config5", "config2", "config4"), default="config3")
    ap.add_argument("--games", type=int, default=None, help="config3: 256; config5: 65536; config4: 8192 (whole job)")
    ap.add_argument("--rollouts", type=int, default=1024)
    ap.add_argument("--iterations", type=int, default=4096, help="config5 MCTS iterations per search")
    ap.add_argument("--chunk", type=int, default=None,
                    help="config5 iterations per launch (default: all of them in one launch; 4,096: 19.03 / "
                         "19.05 M sims/s vs 18.78 / 18.84 M in 1,024-iteration launches, "
                         "profiles/r05/sweeps/r05at: each launch ends with its slowest search)")
    ap.add_argument("--rollout-policy", choices=("random", "heuristic"), default="random",
                    help="config5: RandomAgent rollouts (the workload) or HeuristicAgent rollouts "
                         "(MCTSAgent's default rollout agent)")
    ap.add_argument("--boards", type=int, default=4096, help="config2 boards")
    ap.add_argument("--all-players", action="store_true", help="config2: all 4 players of every board")
    ap.add_argument("--no-graph", action="store_true",
                    help="config2: launch every step from the host instead of replaying a captured hipGraph")
    ap.add_argument("--root-plies", type=int, default=20)
    ap.add_argument("--seed", type=int, default=20260301)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-cores", type=int, default=None,
                    help="config4: host cores this rank may use (default: the usable cores / local ranks; "
                         "each rank's host phases and worker threads are pinned to its own cores)")
    ap.add_argument("--search-streams", type=int, default=None,
                    help="config4: MCTS searches in flight on this many streams while the other games play on "
                         "(ArenaOptions.search_streams, 1..16; default: the driver's 8)")
    ap.add_argument("--handback", action="store_true",
                    help="config4: hand each search's move back as it finishes (ArenaOptions.handback), not when "
                         "its launch ends")
    ap.add_argument("--job-games", type=int, default=None,
                    help="config4: at most this many searches per bk_mcts launch (ArenaOptions.job_games; "
                         "default: one launch per round)")
    ap.add_argument("--hw-queues", type=int, default=16,
                    help="config4: HIP hardware queues of this rank (GPU_MAX_HW_QUEUES, <= 32; default 16), so the "
                         "search streams, the FastMCTS handle and the main stream do not share in-order queues "
                         "(HIP's default is 4); 0 leaves the environment's setting")
    ap.add_argument("--order", choices=("naive", "frontier"), default="frontier",
                    help="config3 in-kernel move order of the line's value: the reference's default frontier order "
                         "(CPython set tables carried per game; default) or naive")
    ap.add_argument("--no-second-order", "--no-naive-order", "--no-frontier-order", dest="no_second_order",
                    action="store_true",
                    help="config3: skip the line's object for the other move order (naive_order / frontier_order)")
    ap.add_argument("--no-extra-configs", action="store_true",
                    help="config3: skip the line's config5 and config4 objects")
    ap.add_argument("--extra-config5-games", type=int, default=65536,
                    help="config3 line's config5 object: searches of the whole job (strong scaling)")
    ap.add_argument("--extra-config5-iterations", type=int, default=4096,
                    help="config3 line's config5 object: MCTS iterations per search (one launch)")
    ap.add_argument("--extra-config4-games", type=int, default=1024,
                    help="config3 line's config4 object: arena games per rank (weak scaling; 8 ranks = 8,192)")
    a = ap.parse_args(argv)
    if a.steps is None:
        a.steps = 1 if a.workload in ("config5", "config4") else (200 if a.workload == "config2" else 20)
    if a.warmup is None:
        a.warmup = 1 if a.workload in ("config5", "config4") else 3
    if a.chunk is None:
        a.chunk = a.iterations
    return a


# ------------------------------------------------------------------ host CPU facts
def host_cpu():
    """Cores this process may really use on this host (affinity, capped by the cgroup
    CPU quota: on the GPU box nproc shows the whole machine) and the CPU model."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, math.floor(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    cores = min(aff, quota) if quota else aff
    return {"cores": cores, "affinity_cpus": aff, "cgroup_quota_cpus": quota, "model": model}


def ref_python(value, per_core, cores, what):
    return {"value_per_core": per_core, "unit": "sims/s", "what": what,
            "where": f"reference Python engine measured in the {REF_CONTAINER} (SURVEY.md 6); "
                     "the reference cannot run on the GPU box",
            "gpu_over_ref_1core": value / per_core, "gpu_over_ref_all_cores": value / (per_core * cores)}


def cpu_baseline_playouts(roots_np, seconds, order, rollouts, seed=None, gpu_out=None, fast_naive=False):
    """oracle/blokus_oracle.c (C restatement of the reference engine) timed on this
    host's cores on a bounded sample of the same workload, in the SAME move order as the
    GPU line, game-over check after every move like the reference.  Naive order: the
    sample is the first playouts of the last timed step -- same roots (root i //
    rollouts), same Philox streams (seed, playout id) -- so the CPU plays exactly the
    GPU's games, and their result records are compared (gpu_out: that step's uint8
    [n, 32] results).  fast_naive: the naive list is built from the frontier set's
    anchors and sorted row-major (OR_ORDER_NAIVE_VIA_FRONTIER, the same list, ~5x faster
    than the 400-anchor scan), so the ratio is against the fastest CPU path the oracle has."""
    from oracle import pyoracle as O
    cpu = host_cpu()
    threads = cpu["cores"]
    o = O.ORDER_NAIVE if order == "naive" else O.ORDER_FRONTIER
    if order == "naive" and fast_naive:
        o = O.ORDER_NAIVE_VIA_FRONTIER
    same = order == "naive" and seed is not None
    st = (O.State * len(roots_np)).from_buffer_copy(roots_np.tobytes())
    kw = dict(threads=threads, order=o)
    if same:
        import numpy as np
        kw.update(rng=O.RNG_PHILOX, root_index=np.arange(len(roots_np) * rollouts, dtype=np.int32) // rollouts)
    n = 8 * threads
    t0 = time.perf_counter()
    O.batch_playouts(st, n, seed if same else 1, **kw)
    dt = time.perf_counter() - t0
    n2 = max(n, int(n * seconds / max(dt, 1e-3)))  # scale the sample to ~`seconds`
    n2 = min(n2, len(roots_np) * rollouts) if same else n2
    t0 = time.perf_counter()
    res = O.batch_playouts(st, n2, seed if same else 2, **kw)
    dt = time.perf_counter() - t0
    out = {"value": n2 / dt, "unit": "sims/s", "cores": threads, "kind": "port", "cpu_model": cpu["model"],
           "host": cpu, "order": order,
           "sample": f"{n2} arena playouts from the same {len(roots_np)} roots, oracle/blokus_oracle.c in "
                     f"{order} move order{' (list from frontier anchors, sorted)' if o == 2 else ''}, "
                     f"{threads} threads (one per usable core), {dt:.1f} s"}
    if same and gpu_out is not None:
        g = gpu_out[:n2].cpu().numpy().tobytes()
        out["sample"] += "; the GPU's own games (same roots and Philox streams as the last timed step)"
        out["same_games_bit_identical"] = g == bytes(res)
    return out


def cpu_baseline_frontier(roots_np, sets_np, seconds, rollouts, seed, gpu_out):
    """The frontier-order config-3 CPU baseline: oracle/blokus_oracle.c plays the GPU's own
    games of the last timed step -- same roots with the same CPython frontier-set tables
    (root i // rollouts), same Philox streams (seed, playout id), the reference's default
    move order -- on this host's cores (one playout per thread at a time; ctypes releases
    the GIL inside or_playout_arena_philox), and compares the result records."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import pyoracle as O
    cpu = host_cpu()
    threads = cpu["cores"]
    # raw clones of the root boards (a Board.copy() would re-lay the set tables out)
    raw = [bytes(O.board_from(roots_np[g].tobytes(), sets_np[g])) for g in range(len(roots_np))]

    def one(pid):
        b = O.Board.from_buffer_copy(raw[pid // rollouts])
        r, _ = O.playout_arena_philox(b, seed, pid, O.ORDER_FRONTIER)
        return bytes(r)

    n = 8 * threads
    with ThreadPoolExecutor(threads) as ex:
        t0 = time.perf_counter()
        list(ex.map(one, range(n)))
        dt = time.perf_counter() - t0
        n2 = min(len(roots_np) * rollouts, max(n, int(n * seconds / max(dt, 1e-3))))
        t0 = time.perf_counter()
        res = list(ex.map(one, range(n2)))
        dt = time.perf_counter() - t0
    g = gpu_out[:n2].cpu().numpy().tobytes()
    return {"value": n2 / dt, "unit": "sims/s", "cores": threads, "kind": "port", "cpu_model": cpu["model"],
            "host": cpu, "order": "frontier",
            "sample": f"the GPU's own first {n2} playouts of the last timed step (same roots and CPython "
                      f"frontier tables, same Philox streams), oracle/blokus_oracle.c in frontier move order, "
                      f"{threads} threads (one per usable core), {dt:.1f} s",
            "same_games_bit_identical": g == b"".join(res)}


def pin_host_cores(k=None):
    """Pin this rank (its current thread, and so every thread it starts later: the arena's
    search worker, the library's host threads) to its own share of the host's cores: k
    cores, default the usable cores / LOCAL_WORLD_SIZE (an 8-rank node leaves each rank
    1/8 of the host).  Returns {"cores": k, "cpus": [...]}."""
    import torch
    cpus = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else []
    local = int(os.environ.get("LOCAL_RANK", "0"))
    nloc = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    if k is None:
        k = max(1, host_cpu()["cores"] // max(1, nloc))
    k = max(1, int(k))
    mine = cpus[local * k:(local + 1) * k] or cpus[:k]
    if mine and hasattr(os, "sched_setaffinity"):
        os.sched_setaffinity(0, mine)
    torch.set_num_threads(k)
    return {"cores": k, "cpus": mine}


# ------------------------------------------------------------------ N-rank launch
def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` run directly (no WORLD_SIZE in the environment): start N rank
    processes of this same script, one per GPU (LOCAL_RANK r -> device r), with the
    torch.distributed env contract of torch.distributed.run, and wait for them.  This
    process never touches the GPU and never execs; rank 0 prints the JSON line on the
    inherited stdout.  If one rank fails the others are stopped (they would wait at
    a barrier forever).  Returns the exit code to use (first failing rank's, else 0).
    This replaces the reference's only parallelism, the process pool over whole games
    (scripts/arena_tuning.py:124-131)."""
    import signal
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = set(range(n))
    while live:
        for r in sorted(live):
            code = procs[r].poll()
            if code is None:
                continue
            live.discard(r)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                print(f"bench.py: rank {r} exited with {code}; stopping the other ranks", file=sys.stderr)
                for q in live:
                    procs[q].send_signal(signal.SIGTERM)
        time.sleep(0.05)
    return rc


def setup(args):
    """Join the job: world size from the process group (RCCL on GPUs, gloo for the
    --selftest), checked against --gpus."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    import torch
    dist = None
    if args.share_device:  # hardware rehearsal of the N-rank path on one GPU (RCCL wants one rank per GPU)
        local = 0
    if not args.selftest:
        torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        if args.selftest or args.share_device:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        got = dist.get_world_size()
        if got != world or (args.gpus is not None and got != args.gpus):
            raise SystemExit(f"bench.py: process group has {got} ranks, expected {args.gpus or world}")
        world, rank = got, dist.get_rank()
    return world, rank, local, dist


def barrier_sync(dist):
    import torch
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()


def reduce_max_sum(dist, dev, tmax, sums):
    import torch
    t = torch.tensor([tmax], dtype=torch.float64, device=dev)
    s = torch.tensor(sums, dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
    return float(t.item()), [float(x) for x in s.tolist()]


def rank_times(dist, dev, t):
    """Every rank's elapsed seconds (all-gathered), in rank order."""
    import torch
    if not dist:
        return [float(t)]
    x = torch.tensor([t], dtype=torch.float64, device=dev)
    parts = [torch.empty_like(x) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, x)
    return [float(p.item()) for p in parts]


def ranks_fields(dist, rank_elapsed, steps, check=None, sha=None):
    """The N-rank self-check of a line: the world size and backend the
    process group reports, per-rank ms_per_step (min / max), the SHA-256 of the gathered
    records in global order, and whether every global index arrived exactly once."""
    ms = [t / steps * 1e3 for t in rank_elapsed]
    out = {"world_size_reported": dist.get_world_size() if dist else 1,
           "backend": dist.get_backend() if dist else None,
           "ms_per_step_min": min(ms), "ms_per_step_max": max(ms), "ms_per_step_by_rank": ms}
    if sha is not None:
        out["records_sha256"] = sha
    if check is not None:
        out.update(check)
    return out


def traffic_for(kernel, units_per_launch):
    """PMC HBM bytes and VALU instructions of ONE launch of `kernel` holding
    `units_per_launch` units of work (playouts, board-players or simulations), from the
    committed per-unit profile summary (profiles/traffic_latest.json, written by
    tools/summarize_prof.py), with the profile it came from; (None, None, None) if no
    profile covers the kernel."""
    tpath = os.path.join(ROOT, "profiles", "traffic_latest.json")
    try:
        per = json.load(open(tpath)).get("kernels", {}).get(kernel)
    except (OSError, ValueError):
        per = None
    if not per or per.get("bytes_per_unit") is None:
        return None, None, None
    valu = per.get("valu_insts_per_unit")
    src = {"pmc": per.get("source"), "stats": per.get("stats"), "unit": per.get("unit"),
           "profiled_units_per_launch": per.get("units_per_launch"), "units_per_launch": units_per_launch,
           "bytes_per_unit": per["bytes_per_unit"], "valu_insts_per_unit": valu}
    return per["bytes_per_unit"] * units_per_launch, (valu * units_per_launch if valu is not None else None), src


def compute_roofline(valu_insts, avg_ms):
    valu_tops = valu_insts * 64 / (avg_ms * 1e-3) / 1e12 if valu_insts else None
    return {"bound": "valu_int32", "achieved": valu_tops, "peak": VALU_PEAK_TOPS, "unit": "Tlane-op/s",
            "frac": valu_tops / VALU_PEAK_TOPS if valu_tops else None, "peak_single_issue": VALU_SINGLE_TOPS,
            "frac_single_issue": valu_tops / VALU_SINGLE_TOPS if valu_tops else None,
            "valu_insts_per_launch": valu_insts}


# ------------------------------------------------------------------ config 3
def _config3_measure(args, order, gpu, plan, dev, dist):
    """W untimed + K timed config-3 steps in one move order on this rank: 256 synthetic
    20-ply roots made on the GPU from the plan's root streams (naive order: bk_advance;
    frontier order: bk_rollout_frontier SEM_ADVANCE, which also builds each root's four
    CPython frontier-set tables), then per step 262,144 arena playouts (k_rollout /
    k_rollout_fr) on the plan's playout streams.  Timed region: barrier + synchronize on
    both sides; HIP events on the launching stream around every launch."""
    import torch

    roots_np, sets_np, n, out, step = _config3_prepare(args, order, gpu, plan, dev)
    stream = torch.cuda.Stream(dev)  # our kernels and the timing events share this stream
    plies_acc = torch.zeros(1, dtype=torch.int64, device=dev)

    def count_plies():
        plies_acc.add_(out[:, 10:12].contiguous().view(torch.int16).to(torch.int64).sum())

    with torch.cuda.stream(stream):
        for k in range(args.warmup):
            step(k)
            count_plies()
        plies_acc.zero_()
        barrier_sync(dist)
        events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.steps)]
        t0 = time.perf_counter()
        for k in range(args.steps):
            events[k][0].record(stream)
            step(1000 + k)
            events[k][1].record(stream)
            count_plies()
        barrier_sync(dist)
        elapsed = time.perf_counter() - t0
    kernel_ms = [a.elapsed_time(b) for a, b in events]
    per_rank = rank_times(dist, dev, elapsed)
    elapsed, (sims, all_plies) = reduce_max_sum(dist, dev, elapsed, [n * args.steps, int(plies_acc.item())])
    return {"elapsed": elapsed, "sims": sims, "plies": all_plies, "kernel_ms": kernel_ms, "out": out,
            "roots_np": roots_np, "sets_np": sets_np, "n": n, "rank_elapsed": per_rank}


def _config3_prepare(args, order, gpu, plan, dev):
    """The plan's roots on the GPU (and, frontier order, their frontier-set tables), the
    output buffer, and step(k): one launch of the plan's playouts with step seed k."""
    import numpy as np
    import torch

    from reinforcementlearning_blokus_amd import _native as N
    from reinforcementlearning_blokus_amd.gpu import empty_state
    games = plan.games
    sets_np = sets = None
    if order == "frontier":
        roots_np, sets_np = gpu.rollout_frontier(empty_state(), N.fset_new(1), games,
                                                 semantics=N.SEM_ADVANCE, rng=N.RNG_PHILOX, seed=plan.seed,
                                                 max_plies=args.root_plies,
                                                 root_index=np.zeros(games, dtype=np.int32),
                                                 stream_base=plan.root_stream_base)
        sets = torch.from_numpy(sets_np.view(np.uint8).reshape(games, -1).copy()).to(dev)
    else:
        roots_np = gpu.advance(empty_state(), games, args.root_plies, seed=plan.seed,
                               root_index=np.zeros(games, dtype=np.int32), stream_base=plan.root_stream_base)
    roots = torch.from_numpy(roots_np.view(np.uint8).reshape(games, 256)).to(dev)
    n = plan.n_playouts
    # game j's rollouts are contiguous (one wave plays 64 rollouts of the same game)
    idx = torch.from_numpy(plan.root_index()).to(dev)
    out = torch.empty((n, 32), dtype=torch.uint8, device=dev)

    def step(k):
        if order == "frontier":
            gpu.rollout_frontier(roots, sets, n, semantics=N.SEM_ARENA, rng=N.RNG_PHILOX, seed=plan.step_seed(k),
                                 root_index=idx, out=out, stream_base=plan.playout_stream_base)
        else:
            gpu.rollout(roots, n, semantics=N.SEM_ARENA, rng=N.RNG_PHILOX, seed=plan.step_seed(k), root_index=idx,
                        out=out, stream_base=plan.playout_stream_base)

    return roots_np, sets_np, n, out, step


def _config3_check_gather(args, order, gpu, m, rank, world, dist, dev):
    """All-gather every rank's last-step records and, on rank 0, compare them with ONE
    launch of the whole job's N x games games (Config3Plan rank 0 of N x games): the
    weak-scaling claim that an N-rank job equals a 1-rank run of its games, checked on
    the device (`--check-gather`).  Returns "ok" or a description of the first mismatch."""
    import torch

    from reinforcementlearning_blokus_amd.shard import gather_blocks
    from reinforcementlearning_blokus_amd.workloads import Config3Plan
    got = gather_blocks(m["out"], rank, world, dist)
    if rank != 0:
        return None
    games = args.games or 256
    _, _, n, out, step = _config3_prepare(args, order, gpu, Config3Plan(args.seed, games * world, args.rollouts, 0),
                                          dev)
    step(1000 + args.steps - 1)
    torch.cuda.synchronize()
    if got.shape != out.shape:
        return f"gathered {tuple(got.shape)} records, one-rank run has {tuple(out.shape)}"
    bad = (got != out).any(dim=1).nonzero().flatten()
    return "ok" if bad.numel() == 0 else f"{bad.numel()} of {n} records differ (first: playout {int(bad[0])})"


def _config3_fields(args, order, m, world):
    """value / roofline / compute_roofline of one config-3 measurement (SURVEY 8(d) bytes:
    256 B state read + write per ply plus the 32 B result, over the HIP-event launch time)."""
    n = m["n"]
    value = m["sims"] / m["elapsed"]
    avg_ms = sum(m["kernel_ms"]) / len(m["kernel_ms"])
    plies_per_sim = m["plies"] / m["sims"]
    bytes_per_sim = 2.0 * STATE_B * plies_per_sim + RESULT_B
    achieved = (n * bytes_per_sim) / (avg_ms * 1e-3) / 1e9
    kname = "k_rollout_fr" if order == "frontier" else "k_rollout"
    traffic, valu_insts, tsrc = traffic_for(kname, n)
    return {
        "value": value, "unit": "sims/s", "ms_per_step": m["elapsed"] / args.steps * 1e3,
        "workload": f"config3: {args.games or 256} concurrent games x {args.rollouts} random rollouts (arena "
                    f"semantics, {order} move order, Philox RNG) from GPU-generated {args.root_plies}-ply positions",
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": kname, "kernel_ms": avg_ms,
                     "plies_per_sim": plies_per_sim, "bytes_per_sim": bytes_per_sim, "traffic_profile": tsrc},
        "compute_roofline": compute_roofline(valu_insts, avg_ms),
    }


def _config3_cpu(args, order, m, plan, value):
    if order == "frontier":
        cb = cpu_baseline_frontier(m["roots_np"], m["sets_np"], args.cpu_seconds, args.rollouts,
                                   plan.step_seed(1000 + args.steps - 1), m["out"])
    else:  # the naive list built the fastest way the oracle has (frontier anchors + sort)
        cb = cpu_baseline_playouts(m["roots_np"], args.cpu_seconds, order, args.rollouts,
                                   seed=plan.step_seed(1000 + args.steps - 1), gpu_out=m["out"], fast_naive=True)
    cb["gpu_over_cpu"] = value / cb["value"]
    cb["reference_python"] = ref_python(value, REF_PY_ARENA_SIMS_PER_CORE, cb["cores"],
                                        "terminal random playout from ply 20, telemetry off")
    return cb


def run_config3(args, world, rank, local, dist):
    """The default line.  Its value is the --order run (default: the reference's default
    frontier order, engine/move_generator.py:261-559 over the CPython frontier sets of
    engine/board.py:315-367, k_rollout_fr); the line also carries the other order's
    measurement on the same plan (seeds, streams, steps) -- `naive_order` (the reference
    with BLOKUS_USE_FRONTIER_MOVEGEN=0, k_rollout) or `frontier_order` -- with its own
    value, roofline and same-games CPU baseline, and (unless --no-extra-configs) the
    config5 and config4 objects (run_extra_configs)."""
    import numpy as np
    import torch

    from reinforcementlearning_blokus_amd.gpu import BlokusGPU
    from reinforcementlearning_blokus_amd.shard import check_indices, gather_blocks, records_sha256
    from reinforcementlearning_blokus_amd.workloads import Config3Plan
    games = args.games or 256
    gpu = BlokusGPU(local)
    dev = torch.device("cuda", local)
    # every stream is a function of the global game index: rank r plays global games
    # r * games .. (r + 1) * games - 1 (workloads.Config3Plan), so the N-rank job's
    # gathered records equal a 1-rank run of the same N * games games
    plan = Config3Plan(args.seed, games, args.rollouts, rank)
    other = "naive" if args.order == "frontier" else "frontier"
    m = _config3_measure(args, args.order, gpu, plan, dev, dist)
    mo = None if args.no_second_order else _config3_measure(args, other, gpu, plan, dev, dist)
    checks, ranks = {}, None
    if dist:
        # RCCL gather of the last step's terminal results (32 B per playout) over xGMI,
        # outside the timed region; rank r's playouts are the global block r
        got = gather_blocks(m["out"], rank, world, dist)
        idx = check_indices(np.arange(plan.first_game, plan.first_game + games), games * world, world, dist)
        ranks = ranks_fields(dist, m["rank_elapsed"], args.steps, idx, records_sha256(got) if rank == 0 else None)
        if mo is not None:
            goto = gather_blocks(mo["out"], rank, world, dist)
            ranks[f"{other}_order"] = ranks_fields(dist, mo["rank_elapsed"], args.steps, None,
                                                   records_sha256(goto) if rank == 0 else None)
        if args.check_gather:
            checks["gather_check"] = _config3_check_gather(args, args.order, gpu, m, rank, world, dist, dev)
            if mo is not None:
                checks[f"{other}_gather_check"] = _config3_check_gather(args, other, gpu, mo, rank, world, dist, dev)
    extras = {} if args.no_extra_configs else run_extra_configs(args, world, rank, local, dist)
    if rank != 0:
        return None
    f = _config3_fields(args, args.order, m, world)
    line = {
        "metric": METRIC, "value": f["value"], "unit": "sims/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": f["ms_per_step"], "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": f["workload"], "games": games, "rollouts_per_game": args.rollouts,
                   "root_plies": args.root_plies, "playouts_per_step": m["n"], "move_order": args.order,
                   "parallelism": f"dp{world} (independent games per rank)"},
        "roofline": f["roofline"], "compute_roofline": f["compute_roofline"],
    }
    line.update(checks)
    if ranks is not None:
        line["ranks"] = ranks
    if args.share_device:
        line["config"]["parallelism"] += f"; rehearsal: {world} ranks share cuda:0 over gloo"
    if not args.no_cpu_baseline and world == 1:
        line["cpu_baseline"] = _config3_cpu(args, args.order, m, plan, f["value"])
    if mo is not None:
        ff = _config3_fields(args, other, mo, world)
        order_txt = {"frontier": "the reference's default (BLOKUS_USE_FRONTIER_MOVEGEN=1): per (piece, orientation), "
                                 "anchors by the CPython iteration rank of the mover's frontier set",
                     "naive": "BLOKUS_USE_FRONTIER_MOVEGEN=0 (engine/move_generator.py:153-259): piece, orientation, "
                              "anchor row-major"}[other]
        fo = {"value": ff["value"], "unit": "sims/s", "ms_per_step": ff["ms_per_step"], "steps": args.steps,
              "warmup": args.warmup, "workload": ff["workload"], "order": order_txt,
              "roofline": ff["roofline"], "compute_roofline": ff["compute_roofline"]}
        if not args.no_cpu_baseline and world == 1:
            fo["cpu_baseline"] = _config3_cpu(args, other, mo, plan, ff["value"])
        line[f"{other}_order"] = fo
    line.update(extras)
    return line


def run_extra_configs(args, world, rank, local, dist):
    """The default line's config5 and config4 objects, run after the
    config-3 measurement on the same ranks: config 5 = one 65,536 x 4,096 search launch of
    the whole job (strong scaling) after a 64-iteration warmup; config 4 = 1,024 arena
    games per rank (weak scaling: 8 ranks play BASELINE's 8,192) after one warm-up batch.
    A failure is recorded in the object (the config-3 line still prints)."""
    import copy
    import traceback

    import torch
    out = {}
    for name, fn, kw in (("config5", run_config5, dict(games=args.extra_config5_games, iterations=args.extra_config5_iterations,
                                                        chunk=args.extra_config5_iterations,
                                                        rollout_policy="random")),
                         ("config4", run_config4, dict(games=args.extra_config4_games * world))):
        sub = copy.copy(args)
        sub.__dict__.update(kw, steps=1, warmup=1, workload=name, check_gather=False)
        try:
            obj = fn(sub, world, rank, local, dist)
        except Exception as e:  # noqa: BLE001 -- reported in the line, never hidden
            obj = {"error": f"{type(e).__name__}: {e}", "traceback": traceback.format_exc()[-2000:]}
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        if rank == 0 and obj is not None:
            for k in ("n_gpus", "higher_is_better", "vs_baseline", "data"):
                obj.pop(k, None)
            out[name] = obj
    return out


# ------------------------------------------------------------------ config 5
def run_config5(args, world, rank, local, dist):
    import numpy as np
    import torch

    from reinforcementlearning_blokus_amd.gpu import BlokusGPU
    from reinforcementlearning_blokus_amd.shard import shard_indices
    from reinforcementlearning_blokus_amd.workloads import MctsBatch, frontier_roots

    from reinforcementlearning_blokus_amd import _native as N
    heur = args.rollout_policy == "heuristic"
    policy = N.MCTS_ROLLOUT_HEURISTIC if heur else N.MCTS_ROLLOUT_RANDOM
    total = args.games or 65536
    gpu = BlokusGPU(local)
    dev = torch.device("cuda", local)
    # the job's games are global indices 0..total-1 (position, rollout seed and zobrist
    # table are functions of the index); rank r searches games r (mod W)
    mine = shard_indices(total, rank, world)
    roots_all, sets_all = frontier_roots(gpu, total, args.root_plies, seed=args.seed, distinct=None)
    roots, sets = roots_all[mine], sets_all[mine]
    batch = MctsBatch(gpu, roots, sets, iterations=args.iterations, seed0=0, index=mine)
    stream = torch.cuda.current_stream(dev)
    kms = []

    def timed_run(stop_after=None):
        kms.clear()
        batch.reset()
        batch.run(chunk=args.chunk, stop_after=stop_after, on_chunk=lambda k: kms.append(gpu.last_kernel_ms()),
                  rollout_policy=policy)

    for _ in range(args.warmup):  # warmup: the first 64 iterations of the same searches
        timed_run(stop_after=64)
    barrier_sync(dist)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        timed_run()
    barrier_sync(dist)
    elapsed = time.perf_counter() - t0
    res = batch.results()
    sims_local = int(res["iterations_run"].sum()) * args.steps
    plies_local = int(res["rollout_plies"].astype(np.int64).sum())
    unc_local = int(((res["status"] & N.MCTS_EUNCERT) != 0).sum())  # heuristic rollouts only
    bad_local = int(((res["status"] & ~np.uint32(N.MCTS_EUNCERT)) != 0).sum())
    ranks = None
    if dist:
        # RCCL gather of the 32-byte search records (bk_mcts_out) over xGMI, after the
        # timed region, in global game order; every game index must arrive exactly once
        from reinforcementlearning_blokus_amd.shard import check_indices, gather_results, records_sha256
        loc = torch.from_numpy(np.ascontiguousarray(res).view(np.uint8).reshape(len(res), -1).copy()).to(dev)
        got = gather_results(loc, total, rank, world, dist)
        ranks = ranks_fields(dist, rank_times(dist, dev, elapsed), args.steps,
                             check_indices(mine, total, world, dist), records_sha256(got) if rank == 0 else None)
    elapsed, (sims, plies, hits, rollouts, unc, bad) = reduce_max_sum(
        dist, dev, elapsed, [sims_local, plies_local * args.steps, int(res["tt_hits"].sum()) * args.steps,
                             int(res["rollouts"].sum()) * args.steps, unc_local, bad_local])
    del stream
    check = None
    if dist and args.check_gather:
        check = _config5_check_gather(args, gpu, batch, policy, mine, roots_all, sets_all, rank, world, dist)
    if rank != 0:
        return None
    value = sims / elapsed
    kernel_ms = sum(kms)  # last step's launches (HIP events per chunk)
    # SURVEY 8(d) bytes: 256 B state read + write per rollout ply + 32 B result per
    # simulation; plus the tree/TT traffic a search cannot avoid: one TT probe (16 B),
    # one node write (24 B) and a root-to-leaf path update per iteration (~2 x 24 B)
    sims_rank0 = int(res["iterations_run"].sum())
    bytes_rank0 = 2.0 * STATE_B * plies_local + (RESULT_B + 16 + 24 + 48) * sims_rank0
    achieved = bytes_rank0 / (kernel_ms * 1e-3) / 1e9
    kname = gpu.last_kernel() or ("k_mcts_h" if heur else "k_mcts")  # bk_mcts picks it by batch size
    # counters per simulation x this line's simulations per launch (its --chunk)
    traffic, valu_insts, tsrc = traffic_for(kname, sims_rank0 / max(1, len(kms)))
    line = {
        "metric": METRIC if not heur else "MCTSAgent (default HeuristicAgent rollouts) simulations/sec",
        "value": value, "unit": "sims/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u32+f64", "data": "synthetic",
        "config": {"workload": f"config5: {total} concurrent MCTSAgent searches x {args.iterations} iterations "
                               f"(UCT, Zobrist TT in HBM, 50-ply {'HeuristicAgent' if heur else 'RandomAgent'} "
                               "rollouts, reference frontier move order, bit-exact) from GPU-generated "
                               f"{args.root_plies}-ply positions",
                   "games": total, "iterations": args.iterations, "chunk": args.chunk,
                   "simulations_per_step": total * args.iterations,
                   "rollout_plies_per_sim": plies / sims, "tt_hit_rate": hits / sims,
                   # searches with a HeuristicAgent draw within 2^-40 of a probability boundary
                   # (BK_MCTS_EUNCERT; 0 = every choice certified equal to the reference's)
                   "uncertified_searches": int(unc) if heur else None,
                   "failed_searches": int(bad),  # any BK_MCTS_E* status but EUNCERT (0 expected)
                   "parallelism": f"dp{world} (games sharded r mod {world})"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": kname,
                     "kernel_ms": kernel_ms, "launches": len(kms), "traffic_profile": tsrc},
        # VALU instructions of one launch of this line's size over the average launch time
        "compute_roofline": compute_roofline(valu_insts, kernel_ms / max(1, len(kms))),
    }
    if check is not None:
        line["gather_check"] = check
    if ranks is not None:
        line["ranks"] = ranks
    if args.share_device:
        line["config"]["parallelism"] += f"; rehearsal: {world} ranks share cuda:0 over gloo"
    if heur:  # no C restatement of the heuristic search to time: the reference's own numbers
        line["reference"] = {"published": {"value": 40.9, "unit": "sims/s", "what": "MCTSAgent (heuristic "
                                           "rollouts, TT), 200 ms/move, MacBook (BASELINE.md)"},
                             "measured_build_container": {"value": 1.1, "unit": "sims/s/core",
                                                          "what": "MCTSAgent default, 30 iterations (BASELINE.md)"},
                             "gpu_over_published": value / 40.9}
        return line
    if not args.no_cpu_baseline and world == 1:
        cb = cpu_baseline_mcts(roots, sets, batch, args.cpu_seconds)
        cb["gpu_over_cpu"] = value / cb["value"]
        cb["reference_python"] = ref_python(value, REF_PY_MCTS_RANDOM_SIMS, cb["cores"],
                                            "MCTSAgent + RandomAgent rollouts, 100 iterations (one search)")
        line["cpu_baseline"] = cb
    return line


def _config5_check_gather(args, gpu, batch, policy, mine, roots_all, sets_all, rank, world, dist):
    """Gather every rank's search records (games r mod W) and, on rank 0, compare them with
    one batch searching all the job's games in one process (`--check-gather`): the
    strong-scaling claim that a sharded job equals a single-process run, on the device.
    Returns "ok" or the record fields that differ."""
    import numpy as np

    from reinforcementlearning_blokus_amd.workloads import MctsBatch
    parts = [None] * world
    dist.all_gather_object(parts, (mine.tolist(), batch.results().tobytes()))
    if rank != 0:
        return None
    total = len(roots_all)
    one = MctsBatch(gpu, roots_all, sets_all, iterations=args.iterations, seed0=0, index=np.arange(total))
    one.run(chunk=args.chunk, rollout_policy=policy)
    ref = one.results()
    got = np.zeros_like(ref)
    seen = np.zeros(total, dtype=bool)
    for idx, raw in parts:
        got[np.asarray(idx, dtype=np.int64)] = np.frombuffer(raw, dtype=ref.dtype)
        seen[np.asarray(idx, dtype=np.int64)] = True
    if not seen.all():
        return f"{int((~seen).sum())} games gathered from no rank"
    if got.tobytes() == ref.tobytes():
        return "ok"
    diff = [f for f in ref.dtype.names if not np.array_equal(got[f], ref[f])]
    return "records differ in " + ", ".join(diff)


def cpu_baseline_mcts(roots, sets, batch, seconds):
    """or_mcts (C restatement of MCTSAgent.select_action, pinned by tests/golden/mcts.json)
    on this host's cores: the same positions, zobrist tables and rollout streams, fewer
    iterations per search (bounded sample)."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import pyoracle as O
    cpu = host_cpu()
    threads = cpu["cores"]
    ztabs = [O.zobrist_table(t) for t in range(len(batch.zobrist_np))]

    def one(g, iters):
        b = O.board_from(roots[g].tobytes(), sets[g])
        m = O.numpy_mt(0)
        m.mt[:] = batch.mt0[g, :624].tolist()
        m.mti = int(batch.mt0[g, 624])
        O.mcts(b, int(batch.players_np[g]), iters, 1.414, 50, ztabs[int(batch.zidx_np[g])], m, O.TT())
        return iters

    def run(n_search, iters):
        t0 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:  # ctypes releases the GIL inside or_mcts
            sims = sum(ex.map(lambda g: one(g, iters), range(n_search)))
        return sims, time.perf_counter() - t0

    iters = 128
    _, dt = run(threads, iters)
    n_search = max(threads, int(threads * seconds / max(dt, 1e-3)))
    n_search = min(n_search, len(roots))
    sims, dt = run(n_search, iters)
    return {"value": sims / dt, "unit": "sims/s", "cores": threads, "kind": "port", "cpu_model": cpu["model"],
            "host": cpu, "order": "frontier",
            "sample": f"{n_search} of the same searches at {iters} iterations each (oracle/blokus_oracle.c "
                      f"or_mcts), {threads} threads (one per usable core), {dt:.1f} s"}


# ------------------------------------------------------------------ config 4
CONFIG4_AGENTS = [
    {"name": "random", "type": "random"},
    {"name": "heuristic", "type": "heuristic"},
    {"name": "mcts", "type": "mcts", "params": {"iterations": 64, "max_rollout_moves": 50}},
    {"name": "fast_mcts", "type": "fast_mcts", "thinking_time_ms": 50,
     "params": {"deterministic_time_budget": True, "iterations_per_ms": 20.0}},
]


def run_config4(args, world, rank, local, dist):
    """Mixed-agent arena (BASELINE.json configs[3]): round-robin seats of RandomAgent,
    HeuristicAgent, MCTSAgent (default heuristic rollouts, 64 iterations/move) and
    FastMCTSAgent (1,000 iterations/move), reference-exact records; games sharded over
    ranks (r mod W), records all-gathered after the timed region."""
    import torch

    from reinforcementlearning_blokus_amd.arena.config import RunConfig
    from reinforcementlearning_blokus_amd.arena.runner import run_games_batched
    from reinforcementlearning_blokus_amd.shard import shard_indices

    total = args.games or 8192
    host = pin_host_cores(args.host_cores)
    cfg = RunConfig.from_dict({"agents": CONFIG4_AGENTS, "num_games": total, "seed": args.seed,
                               "seat_policy": "round_robin"})
    mine = shard_indices(total, rank, world).tolist()
    dev = torch.device("cuda", local)
    def progress(rnd, left, prof):  # a line per round on stderr: long runs show they are alive
        if rnd % 10 == 1:
            print(f"config4 rank {rank}: round {rnd}, {left} games in play, mcts {prof['mcts_s']:.1f} s",
                  file=sys.stderr, flush=True)

    from reinforcementlearning_blokus_amd.mcts.mcts_agent import SEARCH_TOTALS, reset_search_totals
    opts = {} if args.search_streams is None else {"search_streams": args.search_streams}
    if args.job_games is not None:
        opts["job_games"] = args.job_games
    if args.handback:
        opts["handback"] = True
    for _ in range(args.warmup):
        run_games_batched(cfg, mine[:64], device=local, **opts)
    barrier_sync(dist)
    reset_search_totals()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        recs = run_games_batched(cfg, mine, device=local, progress=progress, **opts)
    barrier_sync(dist)
    elapsed = time.perf_counter() - t0
    per_rank = rank_times(dist, dev, elapsed)
    st = dict(SEARCH_TOTALS)
    from reinforcementlearning_blokus_amd.arena.runner import LAST_BATCH_PROFILE
    phases = dict(LAST_BATCH_PROFILE)
    sims = sum(int(r["agent_move_stats"]["mcts"]["total_simulations"] or 0) for r in recs)
    moves = sum(r["moves_made"] for r in recs)
    elapsed, (games, all_sims, all_moves) = reduce_max_sum(dist, dev, elapsed,
                                                           [len(recs) * args.steps, sims * args.steps,
                                                            moves * args.steps])
    check = ranks = None
    if dist:
        from reinforcementlearning_blokus_amd.shard import check_indices, records_sha256
        gathered = [None] * world
        dist.all_gather_object(gathered, [(r["game_index"], r["final_scores"], r["moves_made"]) for r in recs])
        canon = sorted((g[0], [g[1][k] for k in sorted(g[1])], g[2]) for part in gathered for g in part)
        ranks = ranks_fields(dist, per_rank, args.steps, check_indices([r["game_index"] for r in recs], total, world,
                                                                       dist),
                             records_sha256(json.dumps(canon).encode()) if rank == 0 else None)
        if args.check_gather and rank == 0:
            # the sharded job against one process playing all its games (strong scaling)
            one = {r["game_index"]: (r["game_index"], r["final_scores"], r["moves_made"])
                   for r in run_games_batched(cfg, list(range(total)), device=local)}
            got = {g[0]: tuple(g) for part in gathered for g in part}
            bad = sorted(i for i in one if got.get(i) != one[i])
            check = "ok" if not bad and len(got) == total else \
                f"{len(bad)} of {total} games differ ({len(got)} gathered; first {bad[:4]})"
    if rank != 0:
        return None
    # roofline of the dominant kernel, the bk_mcts kernel with the most launch time
    # (k_mcts_coop_h at these batch sizes; bk_mcts picks it by searches per CU): SURVEY
    # 8(d) bytes, 256 B state read + write per rollout ply, plus 120 B per simulation
    # (result, TT probe, node write, path update), over its launches' HIP-event time
    kname, kst = max(st["by_kernel"].items(), key=lambda kv: kv[1]["kernel_ms"]) if st["by_kernel"] else \
        ("k_mcts_coop_h", {"launches": 0, "kernel_ms": float("nan"), "sims": 0, "rollout_plies": 0})
    kms = kst["kernel_ms"] or float("nan")
    mcts_bytes = 2.0 * STATE_B * kst["rollout_plies"] + (RESULT_B + 16 + 24 + 48) * kst["sims"]
    achieved = mcts_bytes / (kms * 1e-3) / 1e9
    traffic, valu_insts, tsrc = traffic_for(kname, kst["sims"] / max(1, kst["launches"]))
    line = {
        "metric": "arena games/sec (Random/Heuristic/MCTS/FastMCTS round-robin, reference-exact records)",
        "value": games / elapsed, "unit": "games/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "u32+f64", "data": "synthetic",
        "config": {"workload": f"config4: {total} arena games, seats {[a['name'] for a in CONFIG4_AGENTS]} "
                               "round-robin, MCTS 64 iterations/move (heuristic rollouts), FastMCTS 1,000 "
                               "iterations/move, lockstep batches (bk_arena_advance + bk_mcts + bk_fastmcts)",
                   "games": total, "mcts_sims_per_s": all_sims / elapsed, "moves_per_s": all_moves / elapsed,
                   "uncertified_heuristic_rank0": phases.get("uncertified_heuristic"),
                   "rank0_phase_seconds": phases, "host_cores_per_rank": host,
                   "search_streams": args.search_streams or 8, "job_games": args.job_games, "pipelined": True,
                   "handback": args.handback,
                   "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "HIP default"),
                   "parallelism": f"dp{world} (games sharded r mod {world})"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": kname, "kernel_ms": kms,
                     "launches": kst["launches"], "mcts_sims": kst["sims"],
                     "rollout_plies_per_sim": kst["rollout_plies"] / max(kst["sims"], 1), "traffic_profile": tsrc,
                     "all_search_kernels": st["by_kernel"]},
        "compute_roofline": compute_roofline(valu_insts, kms / max(1, kst["launches"])),
        "reference_python": {"value": 1.0 / 20.3, "unit": "games/s/core",
                             "what": "a 4-random-agent game with the reference's default telemetry (20.3 s), "
                                     "measured in the build container (SURVEY.md 6); MCTS seats are slower"},
    }
    if check is not None:
        line["gather_check"] = check
    if ranks is not None:
        line["ranks"] = ranks
    if args.share_device:
        line["config"]["parallelism"] += f"; rehearsal: {world} ranks share cuda:0 over gloo"
    if not args.no_cpu_baseline and world == 1:
        cb = cpu_baseline_config4(cfg, args.cpu_seconds, recs)
        cb["gpu_over_cpu"] = line["value"] / cb["value"]
        line["cpu_baseline"] = cb
    return line


def cpu_baseline_config4(cfg, seconds, gpu_recs=None):
    """oracle/blokus_oracle.c or_arena4_game on this host's cores: the first games of the
    same run (seat assignment and agent seeds of game i from the run config, as the GPU
    run derives them), one game per thread at a time, as many as fit in about `seconds`.
    or_arena4_game replays the reference's records (tests/test_oracle_arena.py), so its
    final scores are compared with the GPU run's records of the same games."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import pyoracle as O
    from reinforcementlearning_blokus_amd.arena.config import (agent_seed, game_seed_from_run_seed,
                                                               seat_assignment_for_game)
    cpu = host_cpu()
    threads = cpu["cores"]
    kinds = {a.name: {"random": 0, "heuristic": 1, "mcts": 2, "fast_mcts": 3}[a.type] for a in cfg.agents}

    def game(gi):
        seats = seat_assignment_for_game(cfg.agent_names, gi, game_seed_from_run_seed(cfg.seed, gi), cfg.seat_policy)
        names = [seats[str(p + 1)] for p in range(4)]
        return O.arena4_game([kinds[n] for n in names], [agent_seed(cfg.seed, gi, n) for n in names],
                             CONFIG4_AGENTS[2]["params"]["iterations"], 1000)

    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:  # ctypes releases the GIL inside or_arena4_game
        list(ex.map(game, range(threads)))
    dt1 = time.perf_counter() - t0
    n = max(threads, int(threads * seconds / max(dt1, 1e-3)) // threads * threads)
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        games = list(ex.map(game, range(n)))
    dt = time.perf_counter() - t0
    plies = sum(g[0] for g in games)
    out = {"value": n / dt, "unit": "games/s", "cores": threads, "kind": "port", "cpu_model": cpu["model"],
           "host": cpu, "sample": f"the run's first {n} games ({plies} plies), oracle/blokus_oracle.c "
                                  f"or_arena4_game (MCTS 64 iterations with HeuristicAgent rollouts, FastMCTS 1,000 "
                                  f"iterations), {threads} threads, {dt:.1f} s"}
    if gpu_recs is not None:
        by = {r["game_index"]: r for r in gpu_recs}
        cmp = [gi for gi in range(n) if gi in by]
        out["same_games_compared"] = len(cmp)
        out["same_games_bit_identical"] = all(
            [by[gi]["final_scores"][str(p + 1)] for p in range(4)] == list(games[gi][1]) for gi in cmp)
    return out


# ------------------------------------------------------------------ config 2
def run_config2(args, world, rank, local, dist):
    import numpy as np
    import torch

    from reinforcementlearning_blokus_amd.gpu import BlokusGPU, empty_state

    gpu = BlokusGPU(local)
    dev = torch.device("cuda", local)
    nb = args.boards
    # 4,096 synthetic mid-game boards, plies uniform in 16..40
    rng = np.random.RandomState(args.seed + rank)
    plies = rng.randint(16, 41, size=nb)
    parts = []
    for m in range(16, 41):
        k = int((plies == m).sum())
        if k:
            parts.append(gpu.advance(empty_state(), k, m, seed=args.seed * 41 + m + 1000 * rank,
                                     root_index=np.zeros(k, dtype=np.int32)))
    boards = np.concatenate(parts)
    if args.all_players:
        st = np.repeat(boards, 4)
        pl = np.tile(np.arange(4, dtype=np.uint8), nb)
    else:
        st, pl = boards, (boards["current_player"] & 3).astype(np.uint8)
    n = len(st)
    states = torch.from_numpy(st.view(np.uint8).reshape(n, 256).copy()).to(dev)
    players = torch.from_numpy(pl.copy()).to(dev)
    from reinforcementlearning_blokus_amd import _native as N
    stream = torch.cuda.Stream(dev)
    cnt = torch.empty(n, dtype=torch.int32, device=dev)
    masks = torch.empty((n, N.N_ORIENTS, 7), dtype=torch.int64, device=dev)

    def step():  # one bk_movegen_mask launch into the preallocated outputs
        gpu._stream_from_torch()
        gpu.handle.movegen_mask(states.data_ptr(), players.data_ptr(), n, masks.data_ptr(), cnt.data_ptr(),
                                N.MEM_DEVICE)

    # A step is a ~16 us kernel; launched one by one from Python (ctypes, memset, launch:
    # ~25 us of host time per step) the GPU waits on the host.  The steps are captured
    # into a hipGraph of `per` launches instead (every step still runs the whole batch),
    # and the timed region replays it (--no-graph: one launch per step from the host).
    per = 1 if args.no_graph else max(d for d in range(1, min(10, args.steps) + 1) if args.steps % d == 0)
    with torch.cuda.stream(stream):
        for _ in range(args.warmup):
            step()
        graph = None
        if not args.no_graph:
            stream.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=stream):
                for _ in range(per):
                    step()
            graph.replay()  # one untimed replay
        barrier_sync(dist)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(args.steps // per):
            if graph is not None:
                graph.replay()
            else:
                step()
        e1.record(stream)
        barrier_sync(dist)
        elapsed = time.perf_counter() - t0
    kernel_ms = e0.elapsed_time(e1) / args.steps
    kname = gpu.last_kernel()  # k_movegen_ml (LDS-staged writes) or k_movegen_m (BK_MG_STAGE=0)
    moves = int(cnt.to(torch.int64).sum().item())
    elapsed, (pairs,) = reduce_max_sum(dist, dev, elapsed, [n * args.steps])
    if rank != 0:
        return None
    value = pairs / elapsed
    achieved = n * MOVEGEN_B / (kernel_ms * 1e-3) / 1e9
    traffic, valu_insts, tsrc = traffic_for(kname, n)
    line = {
        "metric": "batched legal-move generation (board-players/s, 20x20, 4p)", "value": value,
        "unit": "board-players/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": f"config2: {nb} synthetic mid-game boards (plies 16..40) x "
                               f"{'all 4 players' if args.all_players else 'player to move'}: dense legal "
                               "masks, 91 x 7 u64 per board-player, + counts (bk_movegen_mask)",
                   "boards": nb, "board_players": n,
                   "legal_moves_per_board_player": moves / n, "us_per_batch": kernel_ms * 1e3,
                   "launch": "host launch per step" if graph is None else f"hipGraph replays of {per} launches",
                   "parallelism": f"dp{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": kname,
                     "kernel_ms": kernel_ms, "bytes_per_board_player": MOVEGEN_B,
                     "bytes_written_per_board_player": 91 * 7 * 8 + 4, "traffic_profile": tsrc},
        "compute_roofline": compute_roofline(valu_insts, kernel_ms),
    }
    if not args.no_cpu_baseline and world == 1:
        line["cpu_baseline"] = cpu_baseline_movegen(st, pl, args.cpu_seconds, value)
    return line


def cpu_baseline_movegen(st, pl, seconds, value):
    """oracle legal-move generation (reference frontier algorithm) on this host's cores."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import pyoracle as O
    cpu = host_cpu()
    threads = cpu["cores"]
    boards = [O.unpack(O.State.from_buffer_copy(st[i].tobytes())) for i in range(len(st))]

    def work(lo, hi):
        for i in range(lo, hi):
            O.legal_moves(boards[i], int(pl[i]), O.ORDER_FRONTIER)
        return hi - lo

    def run(n):
        step = max(1, n // threads)
        spans = [(i, min(n, i + step)) for i in range(0, n, step)]
        t0 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            done = sum(ex.map(lambda s: work(*s), spans))
        return done, time.perf_counter() - t0

    n, dt = run(min(len(boards), 4 * threads))
    n2 = min(len(boards), max(n, int(n * seconds / max(dt, 1e-3))))
    n2, dt = run(n2)
    r = n2 / dt
    return {"value": r, "unit": "board-players/s", "cores": threads, "kind": "port", "cpu_model": cpu["model"],
            "host": cpu, "gpu_over_cpu": value / r,
            "sample": f"{n2} of the same board-players, oracle/blokus_oracle.c frontier movegen, {threads} threads, "
                      f"{dt:.1f} s (ctypes calls; the GIL is released inside)",
            "reference_python": ref_python(value, REF_PY_MOVEGEN_BOARDS_PER_CORE, threads,
                                           "get_legal_moves at ply 20 (boards/s/core)")}


def run_selftest(args, world, rank, local, dist):
    """CPU check of the N-rank path with gloo (no GPU, no kernels), on the same shard /
    seed / gather code the GPU workloads run:
    * config 3 (weak scaling): every rank takes its Config3Plan (the global games, root
      streams and playout streams run_config3 launches with), makes each local playout's
      32-byte record from them, and all-gathers the blocks with shard.gather_blocks;
    * configs 4/5 (a fixed job split r mod W): every rank takes its shard of the game
      indices (shard.shard_indices), makes each game's record from the per-game inputs the
      GPU path derives from the global index (MctsBatch zobrist table, rollout MT state),
      and all-gathers them with shard.gather_results.
    Rank 0 checks both against one process making every record of the whole job."""
    import numpy as np
    import torch

    from reinforcementlearning_blokus_amd.shard import gather_blocks, gather_results, shard_indices
    from reinforcementlearning_blokus_amd.workloads import Config3Plan, mcts_game_inputs
    total = args.games or 1001  # odd: shards of unequal size
    c3_games, c3_rollouts = 5, 7

    def records(idx):
        idx = np.asarray(idx, dtype=np.int64)
        zi, mt = mcts_game_inputs(idx, seed0=args.seed)
        rec = np.zeros((len(idx), 32), np.uint8)
        w = rec.view(np.uint32)
        w[:, 0] = idx
        w[:, 1] = zi
        w[:, 2:6] = mt[:, :4]
        w[:, 6] = mt[:, 624]
        w[:, 7] = np.bitwise_xor.reduce(mt[:, :624], axis=1)
        return rec

    def c3_records(plan, step):
        """What bk_rollout keys each local playout by: its Philox stream id and key, and
        the stream of its root (bk_advance) -- all as run_config3 passes them."""
        rec = np.zeros((plan.n_playouts, 32), np.uint8)
        w = rec.view(np.uint32)
        w[:, 0] = plan.global_playouts()
        w[:, 1] = plan.root_index() + plan.root_stream_base  # the root's Philox stream = global game
        key = plan.step_seed(step)
        w[:, 2], w[:, 3] = key & 0xFFFFFFFF, key >> 32
        w[:, 4] = plan.seed
        return rec

    if os.environ.get("BENCH_SELFTEST_FAIL_RANK") == str(rank):  # failure injection (tests)
        raise SystemExit(3)
    from reinforcementlearning_blokus_amd.shard import check_indices, records_sha256
    t0 = time.perf_counter()
    mine = shard_indices(total, rank, world)
    got = gather_results(torch.from_numpy(records(mine)), total, rank, world, dist) if dist else \
        torch.from_numpy(records(mine))
    plan = Config3Plan(args.seed, c3_games, c3_rollouts, rank)
    c3 = torch.from_numpy(c3_records(plan, 1000))
    c3_got = gather_blocks(c3, rank, world, dist) if dist else c3
    # the N-rank fields the GPU lines carry (ranks_fields), on the same gathers
    ranks = ranks_fields(dist, rank_times(dist, "cpu", time.perf_counter() - t0), 1,
                         check_indices(mine, total, world, dist), records_sha256(got))
    c3_ranks = check_indices(np.arange(plan.first_game, plan.first_game + c3_games), c3_games * world, world, dist)
    if rank != 0:
        return None
    if records_sha256(got) != records_sha256(torch.from_numpy(records(range(total)))):
        raise SystemExit("bench.py --selftest: gathered records' SHA-256 differs from the one-process records'")
    if not np.array_equal(got.numpy(), records(range(total))):
        raise SystemExit("bench.py --selftest: gathered records differ from the one-process records")
    whole = Config3Plan(args.seed, c3_games * world, c3_rollouts, 0)
    if not np.array_equal(c3_got.numpy(), c3_records(whole, 1000)):
        raise SystemExit("bench.py --selftest: gathered config-3 records differ from a one-rank run of the job")
    return {"selftest": "ok", "n_ranks": world, "backend": "gloo" if dist else "none", "games": total,
            "shard_sizes": [len(shard_indices(total, r, world)) for r in range(world)], "ranks": ranks,
            "config3": {"games_per_rank": c3_games, "rollouts": c3_rollouts, "job_playouts": whole.n_playouts,
                        "ranks": c3_ranks}}


def main():
    args = parse()
    n = args.gpus or 1
    if "WORLD_SIZE" not in os.environ and n > 1:
        sys.exit(launch_ranks(n, sys.argv[1:]))
    # config 4 (alone or as the default line's config4 object): its search streams need
    # their own hardware queues, set before the HIP runtime starts (setup imports torch)
    if args.workload == "config4" or (args.workload == "config3" and not args.no_extra_configs):
        if args.hw_queues:
            if not 1 <= args.hw_queues <= 32:
                raise SystemExit("bench.py: --hw-queues must be in 0..32")
            os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    world, rank, local, dist = setup(args)
    run = {"config3": run_config3, "config5": run_config5, "config2": run_config2,
           "config4": run_config4}[args.workload]
    if args.selftest:
        run = run_selftest
    line = run(args, world, rank, local, dist)
    if line is not None:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
