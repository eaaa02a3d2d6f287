#!/bin/bash
# A/B of an environment setting ($ENVSET, e.g. "BK_BLOCKS_PER_CU=2") on a bench line
# (BENCH_ARGS), alternating runs.  Outputs under gpurun_out/$TAG/.
set -u
TAG=${1:-envab}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
step() { local rc=$1; shift; echo "$* rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/base_$i.jsonl 2> $OUT/base_$i.err; step $? base_$i
  env $ENVSET timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/alt_$i.jsonl 2> $OUT/alt_$i.err; step $? alt_$i
done
