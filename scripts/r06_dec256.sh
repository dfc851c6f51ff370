#!/bin/bash
# Round 6 A/B: the register-staged decode with 256-thread, <= 256-row tiles in 40 KB of LDS (four
# workgroups per CU: fury_amd/alt/libfury_row_dec256.so, built with -DFURY_DEC_THREADS=256
# -DFURY_DEC_BUDGET_KB=40) against the default 512 threads / 80 KB (two per CU); bench.py verifies
# the decoded columns.  Alternating runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R06_OUT:-r06d256}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for w in mixed nested; do
    timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/base_${w}_$rep.json 2> $OUT/base_$w.err || { tail -5 $OUT/base_$w.err; exit 1; }
    FURY_ROW_LIB=$PWD/fury_amd/alt/libfury_row_dec256.so timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/alt_${w}_$rep.json 2> $OUT/alt_$w.err || { tail -5 $OUT/alt_$w.err; exit 1; }
    python3 -c "
import json
for t in ('base','alt'):
    d=json.loads(open('$OUT/'+t+'_${w}_$rep.json').read().strip().splitlines()[-1])
    r=d['roofline']; print(t, '$w', d['value'], 'enc', r['encode_ms'], 'dec', r['decode_ms'])"
  done
done
