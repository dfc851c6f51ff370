#!/bin/bash
# Round 2: the counter list of this gfx950 + SQ counters of the variable-length bench kernels
# (one rocprofv3 --pmc pass per set, never combined with tracing, each pass time-limited).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc_var2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || echo "[pmc_var2] list rc=$?"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU"
i=0
for w in ${WORKLOADS:-mixed}; do
  for C in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/${w}_$i -o run --output-format csv \
      -- python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-e2e \
      > $OUT/${w}_$i.log 2>&1 || exit $?
    echo "[pmc_var2] $w pass $i done"
  done
done
