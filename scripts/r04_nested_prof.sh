#!/bin/bash
# Nested engine at 4M depth-3 rows (default engines): rocprofv3 kernel stats, then FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes (never combined with tracing), per kernel dispatch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R04N_OUT:-r04n}
mkdir -p $OUT
export TMPDIR=/tmp
LEG=${R04N_LEG:-'[{"nested_decode":2}]'}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o n --output-format csv -- python3 scripts/ab_generic.py --rows 4000000 --iters 3 --legs "$LEG" > $OUT/stats.log 2>&1 || { tail -5 $OUT/stats.log; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $C -d $OUT/$C -o n --output-format csv -- python3 scripts/ab_generic.py --rows 4000000 --iters 1 --legs "$LEG" > $OUT/$C.log 2>&1 || { tail -5 $OUT/$C.log; exit 1; }
done
echo "[r04n] done"
