#!/bin/bash
# Round-5 GPU session: the new tests first (verbose), then the whole -m gpu suite, smoke, and
# bench lines of the three BASELINE workloads.  Each GPU step has its own time limit; the first
# failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R05_OUT:-r05a}
mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread"
if [ -n "${FIRST:-}" ]; then
  timeout -k 10 600 $T -x -v $FIRST > $OUT/pytest_first.log 2>&1 || { tail -30 $OUT/pytest_first.log; exit 1; }
  tail -3 $OUT/pytest_first.log
fi
if [ "${FULL:-1}" = "1" ]; then
  timeout -k 10 900 $T -m gpu -x -q tests > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
fi
for w in ${BENCH:-struct100 mixed nested}; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 ${BENCH_ARGS:-} > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail -5 $OUT/bench_$w.err; exit 1; }
  echo "[r05] bench $w: $(cut -c1-200 $OUT/bench_$w.json)"
done
echo "[r05] done"
