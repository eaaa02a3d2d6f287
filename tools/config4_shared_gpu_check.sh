#!/bin/bash
# Regression check of the config-4 double hand-out ("BK_MCTS_ELOG"): two
# ranks sharing the GPU, 16 HW queues and 8 search streams each -- the condition under
# which the handle-creation memset on the null stream used to land inside the first
# search launch (6 of 6 runs failed before the fix, profiles/r06/elog) -- 5 times, then
# the multirank + mcts GPU tests.  Run through gpurun from the repo root.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-c4shared}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for i in 1 2 3 4 5; do
  timeout -k 10 150 python -u bench.py --gpus 2 --share-device --no-cpu-baseline --workload config4 --games 24 \
      --steps 2 --warmup 1 --hw-queues 16 > $OUT/FX.$i.jsonl 2> $OUT/FX.$i.err
  rc=$?
  echo "FX run $i rc=$rc" | tee -a $OUT/summary.txt
  if [ $rc -ne 0 ]; then grep -o "failure record {[^}]*}" $OUT/FX.$i.err | head -2 >> $OUT/summary.txt; exit 0; fi
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank_device.py tests/test_gpu_mcts.py -v --timeout 300 \
    --timeout-method thread > $OUT/tests.log 2>&1
echo "tests rc=$?" | tee -a $OUT/summary.txt
