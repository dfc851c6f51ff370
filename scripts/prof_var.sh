#!/bin/bash
# Kernel-level timing of the variable-length workloads: rocprofv3 kernel stats of the bench and
# the in-process A/B legs (scripts/ab_var.py).  Every GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for w in ${WORKLOADS:-mixed nested}; do
  timeout -k 10 300 python scripts/ab_var.py --workload $w > $OUT/ab_$w.log 2>&1 || exit $?
  tail -1 $OUT/ab_$w.log
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$w -o $w --output-format csv \
    -- python3 bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-e2e \
    > $OUT/prof_$w.log 2>&1 || exit $?
  echo "[prof_var] $w done"
done
