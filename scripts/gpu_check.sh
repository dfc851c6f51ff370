#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel stats.  Every GPU step has its
# own time limit; a crash/timeout (exit >= 2 other than pytest's "tests failed" = 1) stops the run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
echo "[gpu_check] $(date) start" | tee $OUT/progress.log
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "[gpu_check] pytest rc=$rc" | tee -a $OUT/progress.log
tail -5 $OUT/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "[gpu_check] smoke rc=$rc" | tee -a $OUT/progress.log; tail -3 $OUT/smoke.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
rc=$?; echo "[gpu_check] bench rc=$rc" | tee -a $OUT/progress.log; tail -3 $OUT/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv \
    -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/prof.log 2>&1
  rc=$?; echo "[gpu_check] rocprof rc=$rc" | tee -a $OUT/progress.log; tail -3 $OUT/prof.log
fi
echo "[gpu_check] $(date) done" | tee -a $OUT/progress.log
