"""N>1 path on CPU: world_size-2 gloo ranks shard games and gather results.

Each rank plays its shard (game index == rank mod 2) of a fixed set of arena playouts
with the oracle standing in for the device (test infrastructure only), gathers the
32-byte result records with shard.gather_results, and rank 0 checks them against one
process playing every game: the sharded run is bit-identical to the single run.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from reinforcementlearning_blokus_amd.shard import gather_results, shard_indices


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _play(indices):
    """Arena playouts of games `indices`: root = position (i mod 8), agent seeds from i."""
    from oracle import pyoracle as O
    from tests.helpers import POS, replay
    recs = []
    for i in indices:
        b = replay(POS[8 + int(i) % 8])
        res, _ = O.playout_arena(b, [int(i) * 4 + k for k in range(4)], O.ORDER_NAIVE)
        recs.append(np.frombuffer(bytes(res), dtype=np.uint8))
    return np.stack(recs) if recs else np.zeros((0, 32), np.uint8)


def _worker(rank, world, port, n_total, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = _play(shard_indices(n_total, rank, world))
        allres = gather_results(torch.from_numpy(mine), n_total, rank, world, dist)
        if rank == 0:
            q.put(allres.numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [7, 8])
def test_gloo_two_ranks_shard_and_gather(n_total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_total, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _play(range(n_total))
    assert np.array_equal(got, ref)


def test_shard_indices_partition():
    for n in (0, 1, 5, 64, 1001):
        for w in (1, 2, 3, 8):
            allidx = np.sort(np.concatenate([shard_indices(n, r, w) for r in range(w)]))
            assert np.array_equal(allidx, np.arange(n))


def _exp_worker(rank, world, port, out_root, q):
    """run_experiment on one gloo rank; the reference's own game records (arena_runs.json)
    stand in for the device play, so the test covers sharding, the gather and the writer."""
    import copy
    import torch.distributed as dist
    from reinforcementlearning_blokus_amd.arena import RunConfig, runner
    from tests.helpers import load_golden
    fx = load_golden("arena_runs.json")
    played = []

    def fake_play(run_config, indices, **kw):
        played.extend(int(i) for i in indices)
        return [copy.deepcopy(fx["games"][int(i)]) for i in indices]

    runner.run_games_gpu = fake_play
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = RunConfig.from_dict(dict(fx["config"], output_root=out_root))
        out = runner.run_experiment(cfg, rank=rank, world=world, dist=dist)
        q.put((rank, played, out.get("run_dir")))
    finally:
        dist.destroy_process_group()


def test_gloo_two_ranks_run_experiment(tmp_path):
    """run_experiment(world=2): each rank plays game index == rank (mod 2); rank 0 gathers
    and writes games.jsonl / summary.json equal to the reference run (arena_runner.py:914-996)."""
    import json
    from tests.helpers import load_golden
    fx = load_golden("arena_runs.json")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exp_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict((r, (played, d)) for r, played, d in (q.get(timeout=300) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0][0] == list(range(0, 16, 2)) and got[1][0] == list(range(1, 16, 2))
    assert got[1][1] is None
    run_dir = got[0][1]
    games = [json.loads(x) for x in open(os.path.join(run_dir, "games.jsonl")).read().splitlines()]
    assert [g["game_index"] for g in games] == list(range(16))
    for g, ref in zip(games, fx["games"]):
        assert g["final_scores"] == ref["final_scores"] and g["seat_assignment"] == ref["seat_assignment"]
    summary = json.load(open(os.path.join(run_dir, "summary.json")))
    assert summary["completed_games"] == 16
    for k in ("win_stats", "wins_by_seat", "score_stats", "pairwise_matchups"):
        assert summary[k] == json.loads(json.dumps(fx["summary"][k]))


# ---------------------------------------------------------------- bench.py N-rank path
def _bench(args, env_extra=None, timeout=300):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, env=env, cwd=root,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_launches_n_ranks_selftest():
    """`bench.py --gpus 2` run directly starts 2 rank processes itself (the driver's N>1
    command without torch.distributed.run); the gloo self-test shards a job's game
    indices, all-gathers the per-game records and rank 0 finds them equal to one
    process's.  Exactly one JSON line comes out (rank 0's)."""
    import json
    r = _bench(["--selftest", "--gpus", "2"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["selftest"] == "ok" and line["n_ranks"] == 2 and line["shard_sizes"] == [501, 500]
    # the N-rank self-check fields every GPU line carries at N > 1 (bench.ranks_fields)
    rk = line["ranks"]
    assert rk["world_size_reported"] == 2 and rk["backend"] == "gloo"
    assert len(rk["ms_per_step_by_rank"]) == 2 and rk["ms_per_step_min"] <= rk["ms_per_step_max"]
    assert rk["every_index_once"] and rk["indices"] == 1001 and rk["missing"] == rk["duplicates"] == 0
    assert len(rk["records_sha256"]) == 64
    assert line["config3"]["ranks"]["every_index_once"] and line["config3"]["ranks"]["indices"] == 10


def test_check_indices_counts_missing_and_duplicates():
    """shard.check_indices: what rank 0 reports when an index is gathered twice or never."""
    from reinforcementlearning_blokus_amd.shard import check_indices, records_sha256, shard_indices
    ok = check_indices(shard_indices(10, 0, 1), 10, 1, None)
    assert ok == {"indices": 10, "every_index_once": True, "missing": 0, "duplicates": 0}
    bad = check_indices([0, 1, 1, 3, 12], 5, 1, None)
    assert bad == {"indices": 5, "every_index_once": False, "missing": 2, "duplicates": 2}
    assert records_sha256(b"abc") == "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"


def test_bench_rejects_gpus_world_mismatch():
    """Under a launcher, --gpus must equal WORLD_SIZE (n_gpus is never misreported)."""
    r = _bench(["--selftest", "--gpus", "2"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)


def test_bench_rank_failure_stops_job():
    """A failing rank makes the launcher stop the others (rank 0 would wait in the gather
    forever) and exit with the failing rank's code."""
    r = _bench(["--selftest", "--gpus", "2"], {"BENCH_SELFTEST_FAIL_RANK": "1"}, timeout=120)
    assert r.returncode == 3 and "rank 1 exited with 3" in r.stderr


def _search_records(indices, iters=24, max_rollout=8, seed0=777):
    """Config-5 searches of global games `indices` on the oracle (standing in for bk_mcts):
    position i % 8 of the golden positions, zobrist table and rollout stream from
    workloads.mcts_game_inputs -- the per-game inputs MctsBatch gives the device."""
    from oracle import pyoracle as O
    from reinforcementlearning_blokus_amd.workloads import mcts_game_inputs
    from tests.helpers import POS, replay
    zi, mt0 = mcts_game_inputs(indices, seed0)
    ztabs = {}
    out = np.zeros((len(indices), 32), np.uint8)
    w = out.view(np.int32)
    for j, i in enumerate(np.asarray(indices).tolist()):
        b = replay(POS[8 + i % 8])
        m = O.numpy_mt(0)
        m.mt[:] = mt0[j, :624].tolist()
        m.mti = int(mt0[j, 624])
        z = ztabs.setdefault(int(zi[j]), O.zobrist_table(int(zi[j])))
        tt = O.TT()
        ref = O.mcts(b, int(b.cur), iters, 1.414, max_rollout, z, m, tt)
        vis = [v for _, v, _ in ref["children"]]
        w[j, :6] = [i, ref["move"], ref["hits"], tt.count, len(vis), max(vis) if vis else -1]
        w[j, 6] = int(sum(t for _, _, t in ref["children"]))
        w[j, 7] = int(m.mti)
    return out


def _mcts_worker(rank, world, port, n_total, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = _search_records(shard_indices(n_total, rank, world))
        allres = gather_results(torch.from_numpy(mine), n_total, rank, world, dist)
        if rank == 0:
            q.put(allres.numpy().copy())
    finally:
        dist.destroy_process_group()


def test_gloo_two_ranks_config5_searches():
    """Config 5 sharded over 2 gloo ranks: each rank searches games index == rank (mod 2)
    with the per-game inputs MctsBatch derives from the global index; the gathered
    results equal one process searching all games."""
    n_total = 9
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mcts_worker, args=(r, 2, port, n_total, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _search_records(range(n_total))
    assert np.array_equal(got, ref)
    assert len(set(ref.view(np.int32)[:, 1].tolist())) > 1  # real, differing searches


def test_bench_roofline_counters_scale_with_launch_size():
    """bench.py rooflines come from per-unit PMC counters (profiles/traffic_latest.json,
    tools/summarize_prof.py) scaled by the line's own units per launch: a launch with
    twice the work is charged twice the bytes and VALU instructions, whatever launch size
    the profile was taken at (config 5's --chunk, config 4's per-round searches)."""
    import json

    import bench
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for kernel, entry in json.load(open(os.path.join(ROOT, "profiles", "traffic_latest.json")))["kernels"].items():
        u = entry["units_per_launch"]
        b1, v1, src = bench.traffic_for(kernel, u)
        b2, v2, _ = bench.traffic_for(kernel, 2 * u)
        assert abs(b1 - entry["bytes_per_launch"]) <= 1e-6 * entry["bytes_per_launch"]
        assert abs(b2 - 2 * b1) <= 1e-6 * b1
        if v1 is not None:
            assert abs(v2 - 2 * v1) <= 1e-6 * v1
        assert src["pmc"] == entry["source"] and os.path.exists(os.path.join(ROOT, entry["source"]))
    assert bench.traffic_for("no_such_kernel", 1) == (None, None, None)
