#!/bin/bash
# Round-4 profile at HEAD: bench line + rocprofv3 kernel stats for the three
# workloads, then HBM traffic (FETCH_SIZE / WRITE_SIZE, separate --pmc passes) for Struct-100
# (with the hbm_probe calibration) and the two variable-length workloads.  Every GPU step has its
# own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04p
mkdir -p $OUT
export TMPDIR=/tmp
for w in ${WORKLOADS:-struct100 mixed nested}; do
  timeout -k 10 240 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline --no-e2e \
    > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail -5 $OUT/bench_$w.err; exit 1; }
  echo "[r04p] bench $w: $(cut -c1-200 $OUT/bench_$w.json)"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_$w -o $w --output-format csv \
    -- python3 bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-e2e \
    > $OUT/prof_$w.log 2>&1 || { tail -5 $OUT/prof_$w.log; exit 1; }
  echo "[r04p] rocprof $w done"
done
if [ -z "${NO_PMC:-}" ]; then
  bash scripts/pmc.sh > $OUT/pmc_struct100.log 2>&1 || { tail -5 $OUT/pmc_struct100.log; exit 1; }
  echo "[r04p] pmc struct100 done"
  bash scripts/pmc_var_traffic.sh > $OUT/pmc_var.log 2>&1 || { tail -5 $OUT/pmc_var.log; exit 1; }
  echo "[r04p] pmc var done"
fi
echo "[r04p] done"
