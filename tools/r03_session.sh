#!/bin/bash
# Round-3 GPU session (via gpurun from the repo root): optional pytest (TESTS, "" = skip),
# then for each workload in WORKLOADS a bench line, a rocprofv3 --kernel-trace --stats
# run and one PMC pass per counter group (PMC=0 skips those).  Every GPU step has its own
# time limit; the script stops at the first failure.  Outputs under gpurun_out/$TAG/.
set -u
TAG=${1:-r03s}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
step() { local rc=$1; shift; echo "$* rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd $R
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python3 -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; step $? pytest
fi
if [ "${SMOKE:-0}" = "1" ]; then
  timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; step $? smoke
fi
cd /tmp && export TMPDIR=/tmp
declare -A ARGS
ARGS[config3]="--steps 5 --warmup 1 --no-cpu-baseline"
ARGS[config3fr]="--order frontier --steps 5 --warmup 1 --no-cpu-baseline"
ARGS[config2]="--workload config2 --steps 50 --warmup 2 --no-cpu-baseline"
ARGS[config5]="--workload config5 --steps 1 --warmup 0 --no-cpu-baseline"
ARGS[config4]="--workload config4 --games 1024 --steps 1 --warmup 0 --no-cpu-baseline"
declare -A BENCH
BENCH[config3]=""
BENCH[config3fr]="--order frontier"
BENCH[config2]="--workload config2"
BENCH[config5]="--workload config5"
BENCH[config4]="--workload config4 --games 1024"
for W in ${WORKLOADS:-}; do
  mkdir -p $OUT/$W
  timeout -k 10 420 python3 $R/bench.py ${BENCH[$W]} ${BENCH_EXTRA:-} > $OUT/$W/bench.jsonl 2> $OUT/$W/bench.err; step $? "bench $W"
  if [ "${PMC:-1}" = "1" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$W/trace -o run --output-format csv -- python3 $R/bench.py ${ARGS[$W]} > $OUT/$W/trace.log 2>&1; step $? "trace $W"
    i=0
    for counters in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS"; do
      i=$((i+1))
      timeout -k 10 300 rocprofv3 --kernel-trace --pmc $counters -d $OUT/$W/pmc$i -o run --output-format csv -- python3 $R/bench.py ${ARGS[$W]} > $OUT/$W/pmc$i.log 2>&1; step $? "pmc $W $counters"
    done
  fi
done
