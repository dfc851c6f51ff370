#!/bin/bash
# Wide flat variable-length schemas (33 fields x 5M rows): wide tests, then timing legs of the
# count + write design (var_wide 1) vs the round-4 look-back tiles (0), and kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${WIDE_OUT:-r05_wide}
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -x -q -m gpu tests/test_device.py -k "wide" tests/test_bounds.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
for w in ${LEGS:-var_wide=1 var_wide=0}; do
  timeout -k 10 300 python scripts/ab_wide.py --rows 5000000 --ncols 33 --no-plan --tune $w > $OUT/ab_$w.json 2>&1 || { tail -5 $OUT/ab_$w.json; exit 1; }
  tail -1 $OUT/ab_$w.json | cut -c 90-400
done
if [ "${PROF:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o wide --output-format csv -- python3 scripts/ab_wide.py --rows 5000000 --ncols 33 --no-plan --iters 5 > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
  find $OUT/prof -name "*kernel_stats.csv" -exec head -12 {} \; | cut -c1-150
fi
