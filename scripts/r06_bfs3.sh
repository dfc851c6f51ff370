#!/bin/bash
# Round 6: tile BFS with LDS-only barriers -- quick oracle check, phases, 4M legs; then the
# nested / wide / bounds tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R06_OUT:-r06g}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tree.py -k "equals_oracle_and_level_engine and nested7" > $OUT/quick.log 2>&1 || { tail -30 $OUT/quick.log; exit 1; }
tail -1 $OUT/quick.log
for t in "" "--tune bfs_threads=64 --tune bfs_rows=64"; do
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
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_tree.py tests/test_fuzz_gpu.py tests/test_bounds.py > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_device.py -k "wide" > $OUT/tests_wide.log 2>&1; rc=$?
tail -3 $OUT/tests_wide.log
exit $rc
