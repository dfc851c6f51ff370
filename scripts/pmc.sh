#!/bin/bash
# HBM traffic counters for the Struct-100 bench kernels, collected per the MI355X guide:
# separate rocprofv3 passes for FETCH_SIZE and WRITE_SIZE (never combined with tracing), plus the
# same counters on tools/hbm_probe's known-byte streaming kernels for calibration.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc
mkdir -p $OUT
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $C -d $OUT/bench_$C -o run --output-format csv \
    -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/bench_$C.log 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --pmc $C -d $OUT/probe_$C -o run --output-format csv \
    -- tools/hbm_probe 855638016 2 > $OUT/probe_$C.log 2>&1 || exit $?
done
python3 scripts/pmc_summarize.py $OUT > $OUT/summary.json && cat $OUT/summary.json
