#!/bin/bash
# Round 6: schemas past the row walk's limits -- tile BFS (nested_decode 4) vs the level engine (1)
# on deep (6-20 levels) and wide (128 / 200 counted nodes) beans; then nested / bounds tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R06_OUT:-r06h}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/ab_deep.py --levels ${LEVELS:-6,9,12,20} --wide ${WIDE:-128,200} --rows ${ROWS:-1000000} --modes 4,1 > $OUT/ab_deep.log 2>&1 || { tail -20 $OUT/ab_deep.log; exit 1; }
grep "^{" $OUT/ab_deep.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_tree.py tests/test_fuzz_gpu.py > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu tests/test_bounds.py > $OUT/tests_bounds.log 2>&1; rc=$?
grep -E "passed|failed|thread_key|assert" $OUT/tests_bounds.log | tail -8
exit $rc
