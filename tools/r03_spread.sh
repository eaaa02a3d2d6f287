#!/bin/bash
# Config-5 lane-spread sweep (via gpurun): bench config5 at BK_MCTS_SPREAD = 1, 2, 4.
set -u
TAG=${1:-spread}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
step() { local rc=$1; shift; echo "$* rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd /tmp && export TMPDIR=/tmp
for S in ${SPREADS:-1 2 4}; do
BK_MCTS_SPREAD=$S timeout -k 10 300 python3 $R/bench.py --workload config5 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench5_s$S.jsonl 2> $OUT/bench5_s$S.err; step $? bench5_s$S
done
