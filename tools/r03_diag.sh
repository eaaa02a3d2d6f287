#!/bin/bash
# Round-3 diagnostic GPU session (via gpurun from the repo root): section timers of the
# frontier-order kernels (tools/sections.py, library built beforehand with --build) and
# stall / memory-instruction PMC passes of the frontier-order config-3 bench.  Every GPU
# step has its own time limit; the script stops at the first failure.
set -u
TAG=${1:-diag}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
step() { local rc=$1; shift; echo "$* rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd $R
if [ "${SECT:-1}" = "1" ]; then
  timeout -k 10 300 python3 -u tools/sections.py > $OUT/sections.jsonl 2> $OUT/sections.err; step $? sections
fi
if [ "${SECT_MCTS:-0}" = "1" ]; then
  timeout -k 10 400 python3 -u tools/sections.py --mcts > $OUT/sections_mcts.jsonl 2> $OUT/sections_mcts.err; step $? sections_mcts
fi
cd /tmp && export TMPDIR=/tmp
ARGS=${PMC_ARGS:---order frontier --steps 2 --warmup 1 --no-cpu-baseline}
i=0
for counters in ${PMC_SETS:-}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc ${counters//,/ } -d $OUT/pmc$i -o run --output-format csv -- python3 $R/bench.py $ARGS > $OUT/pmc$i.log 2>&1; step $? "pmc ${counters}"
done
