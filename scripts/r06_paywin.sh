#!/bin/bash
# Round 6: payload output windows in the walk's write pass -- depth-3 legs (window sizes), the
# 128 / 200 counted-node beans (groups), then the nested / fuzz tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R06_OUT:-r06pw}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u scripts/ab_generic.py --rows 4000000 --iters 3 --legs '[{}, {"walk_skip": 1}, {"walk_out": 65536}, {"walk_out": 24576}]' > $OUT/generic.log 2>&1 || { tail -20 $OUT/generic.log; exit 1; }
grep pieces $OUT/generic.log | cut -c1-230
for t in walk_out=40960 walk_out=65536 walk_skip=1; do
  timeout -k 10 200 python3 -u scripts/ab_deep.py --levels "" --wide 128,200 --rows 1000000 --modes 2 --tune $t > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
  grep "^{" $OUT/ab.log
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_tree.py tests/test_fuzz_gpu.py tests/test_device.py > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
exit $rc
