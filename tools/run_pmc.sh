#!/bin/bash
# PMC passes over a short bench.py run (GPU box only).  Each pass is its own rocprofv3
# run with --kernel-trace only (no sys/runtime trace alongside --pmc).  Counter sets
# are read one per line from stdin.  Usage: bash tools/run_pmc.sh <tag> < sets.txt
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmc}
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $counters -d $OUT/pmc$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/pmc$i.log 2>&1
  rc=$?
  echo "pass $i ($counters) rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
