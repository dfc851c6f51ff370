#!/bin/bash
# Round 6: phase clocks of the row-walk decode under stage geometries, then the bounds / tree /
# fuzz GPU tests of the round's error-path work.  Each GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R06_OUT:-r06c}
mkdir -p $OUT
export TMPDIR=/tmp
R=${ROWS:-4000000}
for t in "" "--tune walk_threads=64 --tune walk_threads_write=64 --tune walk_stage=24576 --tune walk_stage_write=24576 --tune walk_out=0 --tune walk_pool=2048" \
         "--tune walk_threads=128 --tune walk_stage=45056" ; do
  timeout -k 10 240 python3 -u scripts/tree_phases.py --rows $R $t >> $OUT/phases.jsonl 2>> $OUT/phases.err || { tail -5 $OUT/phases.err; exit 1; }
done
cat $OUT/phases.jsonl | tr -d '\n ' | sed 's/}{/}\n{/g'; echo
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_bounds.py tests/test_fuzz_gpu.py tests/test_tree.py > $OUT/tests.log 2>&1; rc=$?
tail -15 $OUT/tests.log
exit $rc
