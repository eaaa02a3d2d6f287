#!/bin/bash
# Round-end check on one GPU box: smoke, config2 benches, then rocprofv3 stats + PMC of
# config3 and config5 (tools/r02_profile.sh); stops at the first failure.
set -u
TAG=${1:-r02_end}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
step() { local rc=$1; shift; echo "$* rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd $R
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; step $? smoke
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --workload config2 > $OUT/bench_config2.jsonl 2> $OUT/bench_config2.err; step $? bench2
cd $R
WORKLOADS="config3 config5" bash tools/r02_profile.sh ${TAG}_prof; step $? profile
