#!/bin/bash
# Round 6: tile BFS v2 (waves take a level's nodes) -- quick oracle check, phases, 4M legs against
# the walk, deep / wide-nested A/B, then the nested / fuzz / bounds tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R06_OUT:-r06i}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tree.py -k "equals_oracle_and_level_engine and nested7" > $OUT/quick.log 2>&1 || { tail -30 $OUT/quick.log; exit 1; }
tail -1 $OUT/quick.log
for t in "--tune nested_decode=4" "--tune nested_decode=4 --tune bfs_threads=256 --tune bfs_rows=128"; do
  timeout -k 10 240 python3 -u scripts/tree_phases.py --rows 4000000 $t >> $OUT/phases.jsonl 2>> $OUT/phases.err || { tail -5 $OUT/phases.err; exit 1; }
done
tr -d '\n ' < $OUT/phases.jsonl | sed 's/}{/}\n{/g'; echo
DEFLEGS='[{}]'
timeout -k 10 600 python3 -u scripts/ab_generic.py --rows 4000000 --iters 3 --legs "${LEGS:-$DEFLEGS}" > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
python3 - $OUT/ab.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if '"pieces_ms"' in l:
        d = json.loads(l); print(d["leg"], d["pieces_ms"], "decode", d["decode_ms"], d["decode_GBps"])
    elif '"equal_to_first"' in l:
        print(l.strip())
PY
timeout -k 10 600 python -u scripts/ab_deep.py --levels 6,9,12,20 --wide 128 --rows 1000000 --modes 4,2,1 > $OUT/ab_deep.log 2>&1 || { tail -20 $OUT/ab_deep.log; exit 1; }
grep "^{" $OUT/ab_deep.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_tree.py tests/test_fuzz_gpu.py > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu tests/test_bounds.py > $OUT/tests_bounds.log 2>&1; rc=$?
grep -E "passed|failed|thread_key|AssertionError" $OUT/tests_bounds.log | tail -8
exit $rc
