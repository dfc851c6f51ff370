#!/bin/bash
# Round 6: tile-BFS phase clocks and legs (after moving row / node bases into LDS), the wide
# plan decode, and the quarantine test.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R06_OUT:-r06f}
mkdir -p $OUT
export TMPDIR=/tmp
for t in "" "--tune bfs_threads=64 --tune bfs_rows=64" "--tune nested_decode=2"; do
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
timeout -k 10 300 python scripts/ab_wide.py --rows 5000000 --ncols 33 --no-plan > $OUT/wide.json 2>&1 || { tail -5 $OUT/wide.json; exit 1; }
tail -1 $OUT/wide.json
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_bounds.py -k quarantine tests/test_device.py -k "wide" > $OUT/tests.log 2>&1; rc=$?
tail -15 $OUT/tests.log
exit $rc
