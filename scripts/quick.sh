#!/bin/bash
# GPU parity tests, then the in-process var A/B timings (each step time-limited; stop at first failure).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for w in ${WORKLOADS:-mixed nested}; do
  timeout -k 10 200 python scripts/ab_var.py --workload $w > gpurun_out/ab_$w.log 2>&1 || exit $?
  tail -n1 gpurun_out/ab_$w.log
done
