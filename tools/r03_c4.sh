#!/bin/bash
# Config-4 session (via gpurun): cProfile of a 1,024-game bench run (host phases), then
# the full 8,192-game single-GPU bench line.  Outputs under gpurun_out/$TAG/.
set -u
TAG=${1:-c4}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
step() { local rc=$1; shift; echo "$* rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -m cProfile -o $OUT/c4_1024.prof $R/bench.py --workload config4 --games 1024 --no-cpu-baseline > $OUT/bench_1024.jsonl 2> $OUT/bench_1024.err; step $? c4_1024
if [ "${FULL:-1}" = "1" ]; then
timeout -k 10 900 python3 $R/bench.py --workload config4 --games 8192 ${FULL_ARGS:-} > $OUT/bench_8192.jsonl 2> $OUT/bench_8192.err; step $? c4_8192
fi
