#!/bin/bash
# A/B of library builds on one box: for each round r in 1..ROUNDS, every variant in
# $VARIANTS ("name=path-to-.so", "base" = the in-tree library) runs `bench.py $ARGS` once,
# alternating, into gpurun_out/$TAG/<name>_<r>.jsonl.  Run through gpurun from the repo root.
set -u
TAG=${1:?tag}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in $VARIANTS; do
    name=${v%%=*}; lib=${v#*=}
    [ "$lib" = base ] && lib=$GRAFT_REPO_ROOT/reinforcementlearning_blokus_amd/_lib/libblokus_hip.so
    BK_LIB_PATH=$lib timeout -k 10 300 python -u bench.py $ARGS > $OUT/${name}_$r.jsonl 2> $OUT/${name}_$r.err
    rc=$?
    echo "$name $r rc=$rc $(grep -o '"value": [0-9.e+]*' $OUT/${name}_$r.jsonl | head -1)" | tee -a $OUT/summary.txt
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
