#!/bin/bash
# k_movegen_g orientation-group sweep (BK_MG_GROUPS) on config 2 (4,096 boards) and its
# all-players variant; "auto" = the library's own choice.  Stops at the first failure.
set -u
TAG=${1:-mg_sweep}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for G in ${GROUPS_LIST:-auto 8 16 24 32 48 64}; do
  for V in "" "--all-players"; do
    if [ "$G" = auto ]; then unset BK_MG_GROUPS; else export BK_MG_GROUPS=$G; fi
    timeout -k 10 120 python3 $R/bench.py --workload config2 $V --no-cpu-baseline --steps 400 > $OUT/g${G}${V}.jsonl 2>/dev/null
    rc=$?; echo "G=$G $V rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
