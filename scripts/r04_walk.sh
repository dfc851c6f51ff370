#!/bin/bash
# Row-walk decode diagnostics at 4M depth-3 rows: phase clocks per tuning leg (WALK_TUNES, one leg
# per line of space-separated key=value pairs), then rocprofv3 kernel stats of the default leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04w
mkdir -p $OUT
export TMPDIR=/tmp
i=0
while IFS= read -r leg; do
  [ -z "$leg" ] && continue
  args=""
  for kv in nested_decode=2 $leg; do args="$args --tune $kv"; done
  timeout -k 10 200 python scripts/tree_phases.py --rows 4000000 $args > $OUT/phases_$i.log 2>&1 || { tail -5 $OUT/phases_$i.log; exit 1; }
  echo "== $leg"; python3 -c "
import json,sys
s=open('$OUT/phases_$i.log').read(); s=s[s.index('{'):]
d=json.loads(s[:s.rindex('}')+1])
for k in ('decode_pass1','decode_pass2'): print(k, d['phases'][k])"
  i=$((i+1))
done <<< "${WALK_TUNES:-walk_stage=49152}"
if [ -n "${PROF:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o walk --output-format csv -- python3 scripts/ab_generic.py --rows 4000000 --iters 3 --legs "${PROF_LEGS:-[{\"nested_decode\":2}]}" > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
  python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/r04w/prof/walk_kernel_stats.csv')))
for r in rows[:16]:
    print(f"{r['Name'][:80]:80s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f}us")
PY
fi
echo "[r04w] done"
