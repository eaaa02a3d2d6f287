#!/bin/bash
# config5 bench (+ CPU baseline) and its rocprofv3 kernel stats, config4 arena bench; stops at the first failure
set -u
TAG=${1:-r02_m}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
step() { local rc=$1; shift; echo "$* rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py --workload config5 > $OUT/bench_config5.jsonl 2>$OUT/bench_config5.err; step $? bench5
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof5 -o run -- python3 $R/bench.py --workload config5 --no-cpu-baseline > $OUT/prof5.log 2>&1; step $? prof5
timeout -k 10 500 python3 $R/bench.py --workload config4 --games ${C4_GAMES:-1024} > $OUT/bench_config4.jsonl 2>$OUT/bench_config4.err; step $? bench4
