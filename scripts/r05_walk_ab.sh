#!/bin/bash
# Nested (depth-3, 4M rows) decode / encode A/B legs plus a kernel-stats profile of the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R05_OUT:-r05w}
mkdir -p $OUT
export TMPDIR=/tmp
ROWS=${ROWS:-4000000}
LEGS=${LEGS:-'[{}]'}
PL=${PROF_LEGS:-'[{}]'}
timeout -k 10 600 python3 -u scripts/ab_generic.py --rows $ROWS --iters 3 --legs "$LEGS" > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
cat $OUT/ab.log | cut -c1-600
if [ "${PROF:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o walk --output-format csv -- python3 scripts/ab_generic.py --rows $ROWS --iters 2 --legs "$PL" > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
  f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1)
  cut -d, -f1-4 "$f" | head -14
fi
echo "[r05w] done"
