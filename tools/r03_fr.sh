#!/bin/bash
# Round-3 frontier-order kernels check (via gpurun from the repo root): frontier / MCTS /
# config-5 parity tests, then bench lines for frontier-order config 3 and config 5 (and
# the same with BK_FR_BLOCKS_PER_CU=2 for an A/B of the occupancy).  Each GPU step under
# its own time limit; stop at the first failure.  Outputs under gpurun_out/$TAG/.
set -u
TAG=${1:-r03fr}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
step() { local rc=$1; shift; echo "$* rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd $R
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests/test_gpu_frontier.py tests/test_gpu_mcts.py tests/test_gpu_p3_replay.py tests/test_gpu_arena.py} -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; step $? pytest
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --order frontier --no-cpu-baseline > $OUT/bench3fr.jsonl 2> $OUT/bench3fr.err; step $? bench3fr
timeout -k 10 300 python3 $R/bench.py --workload config5 --no-cpu-baseline > $OUT/bench5.jsonl 2> $OUT/bench5.err; step $? bench5
if [ "${AB:-1}" = "1" ]; then
BK_FR_BLOCKS_PER_CU=2 timeout -k 10 300 python3 $R/bench.py --order frontier --no-cpu-baseline > $OUT/bench3fr_b2.jsonl 2> $OUT/bench3fr_b2.err; step $? bench3fr_b2
BK_FR_BLOCKS_PER_CU=2 timeout -k 10 300 python3 $R/bench.py --workload config5 --no-cpu-baseline > $OUT/bench5_b2.jsonl 2> $OUT/bench5_b2.err; step $? bench5_b2
fi
