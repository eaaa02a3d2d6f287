#!/bin/bash
# config 5 bench line by launch chunk (iterations per bk_mcts launch)
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/chunks
mkdir -p $OUT
cd /tmp
for c in ${CHUNKS:-512 1024 4096}; do
  timeout -k 10 300 python3 $R/bench.py --workload config5 --chunk $c --steps 1 --warmup 0 --no-cpu-baseline > $OUT/chunk_${c}.jsonl 2> $OUT/chunk_${c}.err
  rc=$?; echo "chunk $c rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
