#!/bin/bash
# coop (4 blocks/CU) vs k_mcts_pair near the random-rollout crossover, 64 iterations
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/cross
mkdir -p $OUT
cd /tmp
for g in 10240 12288; do
for c in 1 0; do
  BK_MCTS_COOP=$c timeout -k 10 300 python3 $R/bench.py --workload config5 --games $g --iterations 64 --chunk 64 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/random_${g}_${c}.jsonl 2> $OUT/random_${g}_${c}.err
  rc=$?; echo "$g coop=$c rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done; done
