#!/bin/bash
# Round-2 measurement session on one GPU box (run via gpurun from the repo root):
#   pytest -m gpu, smoke, and one bench line per workload (config3 default, config2,
#   config2 all players, config5), each step under its own time limit; stops at the
#   first failure.  Outputs under gpurun_out/$TAG/.
set -u
TAG=${1:-r02}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
step() { local rc=$1; shift; echo "$* rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd $R
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; step $? pytest
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; step $? smoke
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py > $OUT/bench_config3.jsonl 2> $OUT/bench_config3.err; step $? bench3
timeout -k 10 300 python3 $R/bench.py --workload config2 > $OUT/bench_config2.jsonl 2> $OUT/bench_config2.err; step $? bench2
timeout -k 10 300 python3 $R/bench.py --workload config2 --all-players > $OUT/bench_config2_all.jsonl 2> $OUT/bench_config2_all.err; step $? bench2all
timeout -k 10 420 python3 $R/bench.py --workload config5 > $OUT/bench_config5.jsonl 2> $OUT/bench_config5.err; step $? bench5
