#!/bin/bash
# heuristic-path GPU tests, heuristic-rollout MCTS bench, config4 bench, movegen group
# sweep; stops at the first failure
set -u
TAG=${1:-r02_h2}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
step() { local rc=$1; shift; echo "$* rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_heuristic.py tests/test_gpu_heuristic_kernel.py tests/test_gpu_arena.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; step $? pytest
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --workload config5 --rollout-policy heuristic --games 65536 --iterations 64 --chunk 64 > $OUT/bench_mcts_heur.jsonl 2>$OUT/bench_mcts_heur.err; step $? bench_heur
timeout -k 10 600 python3 -u $R/bench.py --workload config4 --games ${C4_GAMES:-2048} > $OUT/bench_config4.jsonl 2>$OUT/bench_config4.err; step $? bench4
GROUPS_LIST="auto 8 16 32 48" bash $R/tools/mg_sweep.sh $TAG/mg; step $? mg_sweep
