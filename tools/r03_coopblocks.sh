#!/bin/bash
# k_mcts_coop blocks per CU (random rollouts, 64 iterations) at several batch sizes
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/coopblocks
mkdir -p $OUT
cd /tmp
for g in 2048 4096 8192; do
for b in 2 4; do
  BK_MCTS_COOP=1 BK_COOP_BLOCKS_PER_CU=$b timeout -k 10 300 python3 $R/bench.py --workload config5 --games $g --iterations 64 --chunk 64 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/random_${g}_${b}.jsonl 2> $OUT/random_${g}_${b}.err
  rc=$?; echo "$g bpc=$b rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done; done
