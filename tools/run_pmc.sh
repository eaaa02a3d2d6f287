#!/bin/bash
# PMC passes over tools/prof_target.py (GPU box only).  Each pass is a separate
# rocprofv3 run with --kernel-trace only (no sys/runtime trace alongside --pmc).
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmc}
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $counters -d $OUT/p$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_target.py > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($counters) rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done <<LIST
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_BRANCH
GRBM_GUI_ACTIVE GRBM_COUNT
FETCH_SIZE
WRITE_SIZE
LIST
