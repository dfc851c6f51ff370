#!/bin/bash
# Round 6 A/B: Struct-100 decode variants (tuning fixed_dec: column stores per lane 0 = 8, 1 = 16, 2 = 4; 3 = 8 row loads;
# see fixed.hip), alternating bench.py runs (decoded columns verified).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R06_OUT:-r06fd}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in ${VS:-0 1 2 3}; do
    timeout -k 10 200 python scripts/bench_tuned.py fixed_dec=$v --workload struct100 --steps 30 --warmup 5 --no-cpu-baseline --no-e2e > $OUT/b_${v}_$rep.json 2> $OUT/b_$v.err || { tail -5 $OUT/b_$v.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$OUT/b_${v}_$rep.json').read().strip().splitlines()[-1]); r=d['roofline']
print('fixed_dec=$v', d['value'], 'enc', r['encode_ms'], 'dec', r['decode_ms'], 'copy', r['copy_GBps'])"
  done
done
