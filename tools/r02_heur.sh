#!/bin/bash
# MCTSAgent with heuristic rollouts (k_mcts_h) bench line, then config4 at the full 8,192
# games; stops at the first failure
set -u
TAG=${1:-r02_h}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
step() { local rc=$1; shift; echo "$* rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --workload config5 --rollout-policy heuristic --games 65536 --iterations 64 --chunk 64 > $OUT/bench_mcts_heur.jsonl 2>$OUT/bench_mcts_heur.err; step $? bench_heur
timeout -k 10 900 python3 -u $R/bench.py --workload config4 --games ${C4_GAMES:-8192} > $OUT/bench_config4.jsonl 2>$OUT/bench_config4.err; step $? bench4
