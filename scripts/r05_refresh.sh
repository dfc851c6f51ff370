#!/bin/bash
# Round-5 refresh at HEAD: bench lines for the three workloads (CPU baseline on), a 2-rank
# rehearsal through torch.distributed.run on the one GPU (ranks share it), and rocprofv3 kernel
# stats of each workload.  Each GPU step has its own time limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R05_OUT:-r05f}
mkdir -p $OUT
export TMPDIR=/tmp
for w in struct100 mixed nested; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail -5 $OUT/bench_$w.err; exit 1; }
  echo "[r05 refresh] bench $w: $(cut -c1-160 $OUT/bench_$w.json)"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_$w -o $w --output-format csv \
    -- python3 bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-e2e \
    > $OUT/prof_$w.log 2>&1 || { tail -5 $OUT/prof_$w.log; exit 1; }
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --share-gpus --steps 10 --warmup 2 --no-cpu-baseline --no-e2e \
  > $OUT/bench_2rank.json 2> $OUT/bench_2rank.err || { tail -5 $OUT/bench_2rank.err; exit 1; }
echo "[r05 refresh] 2-rank: $(cut -c1-200 $OUT/bench_2rank.json)"

# the nested 4M depth-3 legs + kernel stats, and the full GPU suite + smoke
R05_OUT=$(basename $OUT)_generic LEGS='[{}]' bash scripts/r05_walk_ab.sh || exit 1
timeout -k 10 900 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu -x -q tests > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
echo "[r05 refresh] all done"
