#!/bin/bash
# Round 6: the persistent two-stage variable-length decode (var_dec_pipe 1 / 2)
# against one tile per workgroup (0) on C3 (mixed) and C4 (nested), outputs checked equal.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R06_OUT:-r06p}
mkdir -p $OUT
export TMPDIR=/tmp
for w in mixed nested; do
  timeout -k 10 300 python -u scripts/ab_dec.py --workload $w --key var_dec_pipe --legs 0,1,2 > $OUT/ab_dec_$w.log 2>&1 || { tail -20 $OUT/ab_dec_$w.log; exit 1; }
  grep "^{" $OUT/ab_dec_$w.log | cut -c1-600
done
