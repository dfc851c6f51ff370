#!/bin/bash
# Deep-schema decode on the row walk (explicit stack): tests, then the walk vs level-engine A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05d
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -x -q -m gpu \
  tests/test_tree.py tests/test_bounds.py tests/test_reference_beans.py > gpurun_out/r05d/tests.log 2>&1 || { tail -30 gpurun_out/r05d/tests.log; exit 1; }
tail -2 gpurun_out/r05d/tests.log
timeout -k 10 600 python -u scripts/ab_deep.py --levels ${LEVELS:-6,9,12,20} --rows ${ROWS:-1000000} > gpurun_out/r05d/ab_deep.log 2>&1 || { tail -20 gpurun_out/r05d/ab_deep.log; exit 1; }
cat gpurun_out/r05d/ab_deep.log
echo "[r05d] done"
