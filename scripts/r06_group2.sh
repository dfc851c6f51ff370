#!/bin/bash
# Round 6: field-group sweep on the 128 / 200 counted-node beans: walk_group_k x prefetch x count
# stage (mode 2 only), then the depth-3 generic schema with small groups.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R06_OUT:-r06g2}
mkdir -p $OUT
export TMPDIR=/tmp
for t in ${SWEEP:-walk_group_k=8 walk_group_k=4 walk_group_k=2 walk_group_k=8,walk_prefetch=0 walk_group_k=4,walk_prefetch=0 walk_group_k=8,walk_stage=0 walk_group_k=4,walk_stage=0,walk_prefetch=0 walk_group_k=8,walk_threads=64}; do
  timeout -k 10 300 python -u scripts/ab_deep.py --levels "" --wide ${WIDE:-128,200} --rows ${ROWS:-1000000} --modes 2 --tune $t > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
  grep "^{" $OUT/ab.log
done
DEFLEGS='[{}, {"walk_group_k": 4}, {"walk_group_k": 2}, {"walk_group_k": 1}]'
timeout -k 10 300 python -u scripts/ab_generic.py --rows 4000000 --legs "${GLEGS:-$DEFLEGS}" > $OUT/generic.log 2>&1 || { tail -20 $OUT/generic.log; exit 1; }
grep "^{" $OUT/generic.log | cut -c1-330
if [ "${PROF:-0}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_counted -o counted -- python scripts/ab_deep.py --levels "" --wide 128 --rows 1000000 --modes 2 > $OUT/prof_counted.log 2>&1 || { tail -5 $OUT/prof_counted.log; exit 1; }
  find $OUT/prof_counted -name '*kernel_stats.csv' -exec cp {} $OUT/counted_kernel_stats.csv \;
  head -6 $OUT/counted_kernel_stats.csv | cut -c1-200
fi
