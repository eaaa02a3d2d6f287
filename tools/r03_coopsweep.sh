#!/bin/bash
# coop vs per-lane MCTS kernels by batch size (heuristic and random rollouts)
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/coopsweep
mkdir -p $OUT
cd /tmp
for pol in heuristic random; do
for g in 8192 16384 32768; do
for c in 1 0; do
  BK_MCTS_COOP=$c timeout -k 10 300 python3 $R/bench.py --workload config5 --rollout-policy $pol --games $g --iterations 64 --chunk 64 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/${pol}_${g}_${c}.jsonl 2> $OUT/${pol}_${g}_${c}.err
  rc=$?; echo "$pol $g coop=$c rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done; done; done
