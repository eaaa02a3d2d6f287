#!/bin/bash
# k_mcts tuning sweep (via gpurun from the repo root): config-5 searches (65,536 games)
# under each setting in SWEEP ("VAR=value ..." groups separated by ';'), one mcts_bench
# line per setting.  Each run has its own time limit; the script stops at the first failure.
set -u
TAG=${1:-tree_sweep}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
IFS=';' read -ra SETS <<< "${SWEEP:-BK_TREE_BATCH=64}"
for s in "${SETS[@]}"; do
  echo "== $s" >> $OUT/sweep.jsonl
  env $s timeout -k 10 200 python3 -u tools/mcts_bench.py --games ${GAMES:-65536} --iterations ${ITERS:-1024} >> $OUT/sweep.jsonl 2>> $OUT/sweep.err
  rc=$?; echo "$s rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
