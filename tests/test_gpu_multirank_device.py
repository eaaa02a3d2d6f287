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


def test_config3_two_ranks_equal_one_launch_of_their_games():
    d = _bench(["--workload", "config3", "--games", "16", "--rollouts", "64", "--steps", "2", "--warmup", "1"])
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["config"]["playouts_per_step"] == 16 * 64
    assert d["gather_check"] == "ok"
    assert d["frontier_gather_check"] == "ok"
    assert "rehearsal" in d["config"]["parallelism"]


def test_config5_two_ranks_equal_one_process():
    d = _bench(["--workload", "config5", "--games", "129", "--iterations", "64", "--chunk", "32",
                "--steps", "1", "--warmup", "1"])
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["gather_check"] == "ok"


def test_config4_two_ranks_equal_one_process():
    d = _bench(["--workload", "config4", "--games", "24", "--steps", "1", "--warmup", "0"], timeout=600)
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["gather_check"] == "ok"
