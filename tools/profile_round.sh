#!/bin/bash
# One GPU-box session of measurements (run via gpurun from the repo root):
#   1. VALU issue-rate probe        -> gpurun_out/$TAG/valu_probe.txt
#   2. bench.py (default, JSON line) -> gpurun_out/$TAG/bench.jsonl
#   3. rocprofv3 --kernel-trace --stats of the bench command -> gpurun_out/$TAG/trace/
#   4. PMC passes FETCH_SIZE / WRITE_SIZE / SQ counters on the same command (one per run)
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
TAG=${1:-prof}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step() { local rc=$1; shift; echo "$* rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
timeout -k 10 120 $R/tools/_bin/valu_probe2 > $OUT/valu_probe2.txt 2>&1; step $? valu_probe2
timeout -k 10 300 python3 $R/bench.py > $OUT/bench.jsonl 2> $OUT/bench.err; step $? bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/trace.log 2>&1; step $? trace
i=0
for counters in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $counters -d $OUT/pmc$i -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc$i.log 2>&1; step $? "pmc $counters"
done
