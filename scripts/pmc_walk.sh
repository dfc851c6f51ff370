#!/bin/bash
# SQ instruction / cycle counters of the row-walk decode kernels (4M depth-3 rows, one leg), one
# --pmc pass (8 SQ counters), never combined with tracing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc_walk
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
  -d $OUT/sq -o run --output-format csv -- python3 scripts/ab_generic.py --rows 4000000 --iters 1 \
  --legs '[{"nested_decode":2}]' > $OUT/sq.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/pmc_walk/sq/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name'][:70]
    if 'walk' not in k and 'rw_' not in k: continue
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, d in acc.items():
    print(k); print('   ', {c: f"{v:.3g}" for c, v in sorted(d.items())})
PY
