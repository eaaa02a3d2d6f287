#!/bin/bash
# Config-4 A/B at 8,192 games: in-tree library vs BK_LIB_PATH=$ALT (no CPU baseline).
set -u
TAG=${1:-c4ab}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
step() { local rc=$1; shift; echo "$* rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py --workload config4 --games ${GAMES:-8192} --no-cpu-baseline > $OUT/base.jsonl 2> $OUT/base.err; step $? base
BK_LIB_PATH=$R/$ALT timeout -k 10 400 python3 $R/bench.py --workload config4 --games ${GAMES:-8192} --no-cpu-baseline > $OUT/alt.jsonl 2> $OUT/alt.err; step $? alt
