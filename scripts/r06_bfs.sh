#!/bin/bash
# Round 6: the tile-BFS nested decode -- a quick oracle check, the 4M depth-3 legs against the row
# walk, then the nested / fuzz / bounds GPU tests.  Each GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R06_OUT:-r06e}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tree.py -k "equals_oracle_and_level_engine and nested7" > $OUT/quick.log 2>&1 || { tail -30 $OUT/quick.log; exit 1; }
tail -1 $OUT/quick.log
DEFLEGS='[{}]'
timeout -k 10 600 python3 -u scripts/ab_generic.py --rows ${ROWS:-4000000} --iters 3 --legs "${LEGS:-$DEFLEGS}" > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
python3 - $OUT/ab.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if '"pieces_ms"' in l:
        d = json.loads(l); print(d["leg"], d["pieces_ms"], "decode", d["decode_ms"], d["decode_GBps"])
    elif '"equal_to_first"' in l:
        print(l.strip())
PY
if [ "${PROF:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o walk --output-format csv -- python3 scripts/ab_generic.py --rows ${ROWS:-4000000} --iters 2 --legs '[{}]' > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
  f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1)
  cut -d, -f1-4 "$f" | head -12
fi
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_tree.py tests/test_fuzz_gpu.py tests/test_bounds.py > $OUT/tests.log 2>&1; rc=$?
  tail -3 $OUT/tests.log
  exit $rc
fi
