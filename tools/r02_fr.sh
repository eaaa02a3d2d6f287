#!/bin/bash
# pytest -m gpu, then the frontier-order benches (config3 --order frontier, config5, heuristic
# MCTS); stops at the first failure.  Outputs under gpurun_out/$TAG/.
set -u
TAG=${1:-r02_fr}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
step() { local rc=$1; shift; echo "$* rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd $R
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; step $? pytest
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --order frontier --no-cpu-baseline > $OUT/bench_config3_fr.jsonl 2> $OUT/bench_config3_fr.err; step $? bench3fr
timeout -k 10 420 python3 $R/bench.py --workload config5 --no-cpu-baseline > $OUT/bench_config5.jsonl 2> $OUT/bench_config5.err; step $? bench5
timeout -k 10 300 python3 $R/bench.py --workload config5 --rollout-policy heuristic --iterations 64 --chunk 64 --no-cpu-baseline > $OUT/bench_mcts_heur.jsonl 2> $OUT/bench_mcts_heur.err; step $? benchheur
