"""The N-rank path of bench.py on a GPU: two rank processes launched by bench.py itself
(launch_ranks), both on the box's one MI355X (`--share-device`: RCCL takes one rank per
GPU, so the rehearsal's process group is gloo), each running its shard through the HIP
kernels, then the gather.  `--check-gather` makes rank 0 replay the whole job in one
process on the device and compare: config 3 (weak scaling: the two ranks' blocks equal
one launch of both ranks' games), config 5 and config 4 (strong scaling: games r mod 2,
with unequal shards).  The CPU suite checks the same launch / shard / gather code on gloo
without a GPU (test_multirank.py); this is the same claim with the kernels in the loop and
two processes sharing the device concurrently."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _bench(args, timeout=420):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, "-u", BENCH, "--gpus", "2", "--share-device", "--check-gather",
                        "--no-cpu-baseline"] + list(args),
                       capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=env)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]  # rank 0 prints the one line
    return json.loads(lines[0])


def _ranks_ok(rk, n_indices):
    """The N-rank self-check fields (bench.ranks_fields): the group's world size, per-rank
    step times, the gathered records' SHA-256, every global index exactly once."""
    assert rk["world_size_reported"] == 2 and rk["backend"] == "gloo"
    assert len(rk["ms_per_step_by_rank"]) == 2 and 0 < rk["ms_per_step_min"] <= rk["ms_per_step_max"]
    assert len(rk["records_sha256"]) == 64
    assert rk["every_index_once"] and rk["indices"] == n_indices


def test_config3_two_ranks_equal_one_launch_of_their_games():
    d = _bench(["--workload", "config3", "--games", "16", "--rollouts", "64", "--steps", "2", "--warmup", "1",
                "--no-extra-configs"])
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["config"]["playouts_per_step"] == 16 * 64 and d["config"]["move_order"] == "frontier"
    assert d["gather_check"] == "ok"
    assert d["naive_gather_check"] == "ok"
    assert "rehearsal" in d["config"]["parallelism"]
    _ranks_ok(d["ranks"], 32)
    assert len(d["ranks"]["naive_order"]["records_sha256"]) == 64


def test_default_line_extra_configs_two_ranks():
    """The default line's config5 / config4 objects at N = 2 (small sizes): each carries
    its own value and the N-rank fields; no error recorded."""
    d = _bench(["--workload", "config3", "--games", "8", "--rollouts", "64", "--steps", "1", "--warmup", "1",
                "--no-second-order", "--extra-config5-games", "66", "--extra-config5-iterations", "64",
                "--extra-config4-games", "6"], timeout=600)
    for name, n in (("config5", 66), ("config4", 12)):
        o = d[name]
        assert "error" not in o, o.get("traceback")
        assert o["value"] > 0 and o["ms_per_step"] > 0 and "roofline" in o
        _ranks_ok(o["ranks"], n)
    assert d["config5"]["config"]["failed_searches"] == 0


def test_config5_two_ranks_equal_one_process():
    d = _bench(["--workload", "config5", "--games", "129", "--iterations", "64", "--chunk", "32",
                "--steps", "1", "--warmup", "1"])
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["gather_check"] == "ok"
    _ranks_ok(d["ranks"], 129)


def test_config4_two_ranks_equal_one_process():
    d = _bench(["--workload", "config4", "--games", "24", "--steps", "1", "--warmup", "0"], timeout=600)
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["gather_check"] == "ok"
    _ranks_ok(d["ranks"], 24)
