#!/bin/bash
# Cooperative frontier walk A/B (via gpurun): coop-kernel parity tests with the walk on and
# off, section shares of both, then the 1,024-game config-4 line.  Outputs under
# gpurun_out/$TAG/.
set -u
TAG=${1:-walk}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
step() { local rc=$1; shift; echo "$* rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd $R
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mcts_coop.py tests/test_gpu_arena.py tests/test_gpu_mcts.py > $OUT/pytest_walk1.log 2>&1; step $? tests_walk1
BK_COOP_WALK=0 timeout -k 10 200 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mcts_coop.py > $OUT/pytest_walk0.log 2>&1; step $? tests_walk0
for w in ${WALKS:-0 1}; do
BK_COOP_WALK=$w timeout -k 10 200 python3 tools/sections.py --coop > $OUT/coop_walk$w.jsonl 2> $OUT/coop_walk$w.err; step $? sections_walk$w
done
cd /tmp && export TMPDIR=/tmp
for w in ${WALKS:-0 1}; do
BK_COOP_WALK=$w timeout -k 10 300 python3 $R/bench.py --workload config4 --games 1024 --no-cpu-baseline > $OUT/c4_walk$w.jsonl 2> $OUT/c4_walk$w.err; step $? c4_walk$w
done
