#!/bin/bash
# Pipelined register encode: var tests, then tuning A/B on mixed (C3) and nested (C4); the walk
# A/B legs first when WALK=1.  (Record of the round-5 experiment, DESIGN §4d: the pipelined encode
# and its tuning "var_enc_pipe" were removed after it measured slower, so this no longer runs.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${WALK:-1}" = "1" ]; then
  PROF=0 R05_OUT=r05w bash scripts/r05_walk_ab.sh || exit 1
fi
timeout -k 10 600 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -x -q -m gpu \
  tests/test_var_lists.py tests/test_device.py tests/test_bounds.py tests/test_config_size.py > gpurun_out/encpipe_tests.log 2>&1 || { tail -30 gpurun_out/encpipe_tests.log; exit 1; }
tail -2 gpurun_out/encpipe_tests.log
bash scripts/ab_tune.sh encpipe "mixed" var_enc_pipe=0 var_enc_pipe=1 var_enc_pipe=2 var_enc_pipe=3 || exit 1
bash scripts/ab_tune.sh encpipe_nested "nested" var_enc_pipe=0 var_enc_pipe=1 || exit 1
echo "[encpipe] done"
