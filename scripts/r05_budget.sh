#!/bin/bash
# Walk item budget: nested tests, then the 4M depth-3 timing + kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05b
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -x -q -m gpu \
  tests/test_tree.py tests/test_bounds.py tests/test_host_fuzz.py tests/test_reference_beans.py > gpurun_out/r05b/tests.log 2>&1 || { tail -30 gpurun_out/r05b/tests.log; exit 1; }
tail -2 gpurun_out/r05b/tests.log
R05_OUT=r05b LEGS='[{}]' bash scripts/r05_walk_ab.sh || exit 1
