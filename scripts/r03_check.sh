#!/bin/bash
# Round-3 GPU session: full GPU test suite, then the bench on the three workloads (short runs,
# no CPU baseline / e2e) -- every step under its own time limit, stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
for w in struct100 mixed nested; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline --no-e2e \
    > $OUT/bench_$w.json 2> $OUT/bench_$w.err
  rc=$?; echo "bench $w rc=$rc"; cat $OUT/bench_$w.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['encode_ms'], d['roofline']['decode_ms'])"
  if [ $rc -ne 0 ]; then tail -5 $OUT/bench_$w.err; exit $rc; fi
done
