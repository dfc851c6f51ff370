#!/bin/bash
# HBM traffic of the variable-length kernels (C3 mixed, C4 nested bench workloads): FETCH_SIZE and
# WRITE_SIZE in separate rocprofv3 --pmc passes (never combined with tracing), summarised per
# launch by scripts/pmc_var_summarize.py with the gfx950 corrections calibrated in
# profiles/pmc_struct100.json (FETCH x2, WRITE x1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc_traffic
mkdir -p $OUT
export TMPDIR=/tmp
for w in ${WORKLOADS:-mixed nested}; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $C -d $OUT/${w}_$C -o run --output-format csv \
      -- python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-e2e \
      > $OUT/${w}_$C.log 2>&1 || exit $?
    echo "[pmc_var_traffic] $w $C done"
  done
  python3 scripts/pmc_var_summarize.py $OUT $w > $OUT/pmc_$w.json || exit $?
done
