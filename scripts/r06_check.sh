#!/bin/bash
# Round 6: targeted GPU tests (error paths, fuzz parity, nested engines) + a headline bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R06_OUT:-r06d}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_bounds.py tests/test_fuzz_gpu.py tests/test_tree.py} > $OUT/tests.log 2>&1; rc=$?
grep -E "^seed|passed|failed|Error" $OUT/tests.log | tail -40
[ $rc = 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline'])"
