#!/bin/bash
# pytest -m gpu + config3 (naive, frontier) + config5 benches; stops at the first failure
set -u
TAG=${1:-r02_q}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
step() { local rc=$1; shift; echo "$* rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; step $? pytest
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline > $OUT/bench_config3.jsonl 2>/dev/null; step $? bench3
timeout -k 10 300 python3 $R/bench.py --order frontier --no-cpu-baseline > $OUT/bench_config3_fr.jsonl 2>/dev/null; step $? bench3fr
timeout -k 10 420 python3 $R/bench.py --workload config5 --no-cpu-baseline > $OUT/bench_config5.jsonl 2>/dev/null; step $? bench5
