#!/bin/bash
# Round-6 refresh at HEAD: bench lines of the three workloads (CPU baseline on), rocprofv3 kernel
# stats of each, a 2-rank rehearsal on the one GPU, the nested 4M legs (+ kernel stats), the wide
# 33 x 5M legs, the deep / wide-nested A/B, then the full GPU suite + smoke.  Each GPU step has its
# own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R06_OUT:-r06r}
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${BENCH:-1}" = "1" ]; then
for w in struct100 mixed nested; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail -5 $OUT/bench_$w.err; exit 1; }
  echo "[r06] bench $w: $(cut -c1-160 $OUT/bench_$w.json)"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_$w -o $w --output-format csv \
    -- python3 bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-e2e \
    > $OUT/prof_$w.log 2>&1 || { tail -5 $OUT/prof_$w.log; exit 1; }
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --share-gpus --steps 10 --warmup 2 --no-cpu-baseline --no-e2e \
  > $OUT/bench_2rank.json 2> $OUT/bench_2rank.err || { tail -5 $OUT/bench_2rank.err; exit 1; }
echo "[r06] 2-rank: $(cut -c1-200 $OUT/bench_2rank.json)"
fi
if [ "${LEGS_RUN:-1}" = "1" ]; then
DEFLEGS='[{}, {"nested_decode":4}]'
timeout -k 10 600 python3 -u scripts/ab_generic.py --rows 4000000 --iters 3 --legs "${LEGS:-$DEFLEGS}" > $OUT/generic_legs.log 2>&1 || { tail -20 $OUT/generic_legs.log; exit 1; }
grep pieces $OUT/generic_legs.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_generic -o walk --output-format csv -- python3 scripts/ab_generic.py --rows 4000000 --iters 2 --legs '[{}]' > $OUT/prof_generic.log 2>&1 || { tail -5 $OUT/prof_generic.log; exit 1; }
timeout -k 10 300 python scripts/ab_wide.py --rows 5000000 --ncols 33 --no-plan > $OUT/wide.json 2>&1 || { tail -5 $OUT/wide.json; exit 1; }
tail -1 $OUT/wide.json | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_wide -o wide --output-format csv -- python3 scripts/ab_wide.py --rows 5000000 --ncols 33 --no-plan --iters 5 > $OUT/prof_wide.log 2>&1 || { tail -5 $OUT/prof_wide.log; exit 1; }
timeout -k 10 600 python -u scripts/ab_deep.py --levels 6,9,12,20 --wide 128,200 --rows 1000000 --modes 3,2,1 > $OUT/deep.log 2>&1 || { tail -20 $OUT/deep.log; exit 1; }
grep "^{" $OUT/deep.log
fi
if [ "${TESTS:-1}" = "1" ]; then
timeout -k 10 1100 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu -x -q tests > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
fi
echo "[r06 refresh] all done"
