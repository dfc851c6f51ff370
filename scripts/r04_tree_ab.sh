#!/bin/bash
# Tree-engine check + A/B at 4M depth-3 rows: tree tests first (stop on failure), phase times,
# then legs of tunings (LEGS env, JSON) timed in one process, then (PROF=1) rocprofv3 stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04t
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_tree.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python scripts/tree_phases.py --rows 4000000 > $OUT/phases.log 2>&1 || { tail -5 $OUT/phases.log; exit 1; }
grep -v amdgpu.ids $OUT/phases.log
LEGS=${LEGS:-'[{"nested_encode":1,"nested_decode":1},{"nested_encode":0,"nested_decode":0}]'}
timeout -k 10 400 python scripts/ab_generic.py --rows 4000000 --legs "$LEGS" > $OUT/ab.log 2>&1 || { tail -5 $OUT/ab.log; exit 1; }
grep -v amdgpu.ids $OUT/ab.log | grep pieces
if [ -n "${PROF:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o tree --output-format csv -- python3 scripts/ab_generic.py --rows 4000000 --iters 2 --legs '[{"nested_encode":0,"nested_decode":0}]' > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
fi
echo "[r04t] done"
