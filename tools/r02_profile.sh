#!/bin/bash
# Round-2 profiling session on one GPU box (run via gpurun from the repo root):
# rocprofv3 --kernel-trace --stats of each bench workload, then one PMC pass per counter
# group (FETCH_SIZE / WRITE_SIZE / SQ) per workload, with the bench's own launches (config5:
# 65,536 x 4,096 iterations in 8 launches, no warm-up step).  WORKLOADS selects workloads.
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
TAG=${1:-r02_prof}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
step() { local rc=$1; shift; echo "$* rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
declare -A ARGS
ARGS[config3]="--steps 5 --warmup 1 --no-cpu-baseline"
ARGS[config3fr]="--order frontier --steps 5 --warmup 1 --no-cpu-baseline"
ARGS[config2]="--workload config2 --steps 50 --warmup 2 --no-cpu-baseline"
ARGS[config5]="--workload config5 --steps 1 --warmup 0 --no-cpu-baseline"
ARGS[config4]="--workload config4 --games 1024 --steps 1 --warmup 0 --no-cpu-baseline"
for W in ${WORKLOADS:-config3 config2 config5}; do
  mkdir -p $OUT/$W
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$W/trace -o run --output-format csv -- python3 $R/bench.py ${ARGS[$W]} > $OUT/$W/trace.log 2>&1; step $? "trace $W"
  i=0
  for counters in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $counters -d $OUT/$W/pmc$i -o run --output-format csv -- python3 $R/bench.py ${ARGS[$W]} > $OUT/$W/pmc$i.log 2>&1; step $? "pmc $W $counters"
  done
done
