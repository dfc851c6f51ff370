#!/bin/bash
# Round 6: field groups of the row walk (walk_group_k) on wide beans (128 / 200 counted nodes) vs
# the level engine, the depth-3 generic legs (no change expected: 1 group), then the nested /
# fuzz / bounds tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R06_OUT:-r06g}
mkdir -p $OUT
export TMPDIR=/tmp
for gk in ${GKS:-16 8 32 0}; do
  timeout -k 10 300 python -u scripts/ab_deep.py --levels "" --wide ${WIDE:-128,200} --rows ${ROWS:-1000000} --modes 2,1 --tune walk_group_k=$gk > $OUT/ab_group_$gk.log 2>&1 || { tail -20 $OUT/ab_group_$gk.log; exit 1; }
  grep "^{" $OUT/ab_group_$gk.log
done
if [ "${LEGS_RUN:-1}" = 1 ]; then
  timeout -k 10 300 python -u scripts/ab_generic.py --rows 4000000 --legs '[{}]' > $OUT/generic.log 2>&1 || { tail -20 $OUT/generic.log; exit 1; }
  grep "^{" $OUT/generic.log | cut -c1-400
fi
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_tree.py tests/test_fuzz_gpu.py > $OUT/tests.log 2>&1; rc=$?
  tail -3 $OUT/tests.log
  [ $rc = 0 ] || exit $rc
  timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu tests/test_bounds.py > $OUT/tests_bounds.log 2>&1; rc=$?
  grep -E "passed|failed|thread_key|assert" $OUT/tests_bounds.log | tail -8
  exit $rc
fi
