#!/bin/bash
# Round-end style refresh: parity tests, smoke, the three bench lines (struct100 headline with
# cpu_baseline + e2e, mixed, nested) and rocprofv3 kernel stats of each.  Every GPU step has its
# own time limit and the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -20 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
for w in struct100 mixed nested; do
  timeout -k 10 300 python bench.py --workload $w > $OUT/bench_$w.log 2>&1 || { tail -5 $OUT/bench_$w.log; exit 1; }
  tail -1 $OUT/bench_$w.log
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$w -o $w --output-format csv \
    -- python3 bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-e2e \
    > $OUT/prof_$w.log 2>&1 || exit $?
done
echo "[refresh] done"
