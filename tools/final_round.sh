#!/bin/bash
# Round-end measurement session on one GPU box (run via gpurun from the repo root):
#   1. pytest -m gpu                       -> gpurun_out/$TAG/pytest_gpu.log
#   2. __graft_entry__.smoke()             -> gpurun_out/$TAG/smoke.log
#   3. bench.py (default, JSON line)       -> gpurun_out/$TAG/bench.jsonl
#   4. rocprofv3 --kernel-trace --stats    -> gpurun_out/$TAG/trace/
#   5. PMC passes FETCH_SIZE, WRITE_SIZE, SQ_* -> gpurun_out/$TAG/pmc{1,2,3}/ (one set per run)
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
TAG=${1:-final}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
step() { local rc=$1; shift; echo "$* rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; step $? pytest
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1; step $? smoke
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py > $OUT/bench.jsonl 2> $OUT/bench.err; step $? bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/trace.log 2>&1; step $? trace
i=0
for counters in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $counters -d $OUT/pmc$i -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc$i.log 2>&1; step $? "pmc $counters"
done
