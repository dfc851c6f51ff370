#!/bin/bash
# Round-4 GPU session: the full GPU test suite (stop on a fault / timeout), then the profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
if [ -n "${NO_PROFILE:-}" ]; then exit $rc; fi
bash scripts/r04_profile.sh
