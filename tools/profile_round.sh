#!/bin/bash
# Profiling session on one GPU box (run via gpurun from the repo root):
#   for each workload in $WORKLOADS (default: config3 config3fr config2 config5 config4):
#   1. rocprofv3 --kernel-trace --stats of the bench command -> gpurun_out/$TAG/<w>/trace/
#   2. one PMC pass per counter group (FETCH_SIZE / WRITE_SIZE / SQ_*), each its own
#      rocprofv3 run with --kernel-trace only (never with sys/runtime traces)
# Then, in the build container: python tools/summarize_prof.py gpurun_out/$TAG/<w> \
#   r05/<name> <kernel> --units <units per launch> --unit <unit> [--keep-first]
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
TAG=${1:-prof}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
step() { local rc=$1; shift; echo "$* rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
declare -A ARGS
ARGS[config3]="--order naive --steps 5 --warmup 1 --no-cpu-baseline --no-second-order --no-extra-configs"
ARGS[config3fr]="--order frontier --steps 5 --warmup 1 --no-cpu-baseline --no-second-order --no-extra-configs"
ARGS[config2]="--workload config2 --steps 50 --warmup 2 --no-cpu-baseline"
ARGS[config5]="--workload config5 --steps 1 --warmup 0 --no-cpu-baseline"
ARGS[config4]="--workload config4 --games 1024 --steps 1 --warmup 0 --no-cpu-baseline"
for W in ${WORKLOADS:-config3 config3fr config2 config5 config4}; do
  mkdir -p $OUT/$W
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$W/trace -o run --output-format csv -- python3 $R/bench.py ${ARGS[$W]} > $OUT/$W/trace.log 2>&1; step $? "trace $W"
  i=0
  for counters in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $counters -d $OUT/$W/pmc$i -o run --output-format csv -- python3 $R/bench.py ${ARGS[$W]} > $OUT/$W/pmc$i.log 2>&1; step $? "pmc $W $counters"
  done
done
