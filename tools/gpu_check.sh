#!/bin/bash
# One validation + A/B session on a GPU box (run via gpurun from the repo root):
# GPU tests, smoke, then the bench lines named in $LINES ("name|env|bench args" per
# line, stdin) into gpurun_out/$TAG/.  Every GPU step has its own time limit; the script
# stops at the first failure.
set -u
TAG=${1:-check}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
step() { local rc=$1; shift; echo "$* rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; step $? tests
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; step $? smoke
fi
while IFS='|' read -r name envs args; do
  [ -z "$name" ] && continue
  env $envs timeout -k 10 300 python bench.py $args > $OUT/$name.jsonl 2> $OUT/$name.err; step $? "bench $name"
done
