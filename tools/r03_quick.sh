#!/bin/bash
# Round-3 quick GPU check (run via gpurun from the repo root): the named pytest files
# (TESTS, default the P3 replay + MCTS tests) then one default bench line; each GPU step
# under its own time limit, stop at the first failure.  Outputs under gpurun_out/$TAG/.
set -u
TAG=${1:-r03q}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
step() { local rc=$1; shift; echo "$* rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd $R
timeout -k 10 600 python3 -u -m pytest ${TESTS:-tests/test_gpu_p3_replay.py tests/test_gpu_mcts.py} -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; step $? pytest
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py ${BENCH_ARGS:-} > $OUT/bench.jsonl 2> $OUT/bench.err; step $? bench
