#!/bin/bash
# Texture-address / texture-data / L1 counters of the variable-length decode (ab_dec.py, one leg),
# one rocprofv3 --pmc pass per set; lists the available counters first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${PMC_OUT:-pmc_ta}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
W=${W:-mixed}
LEG=${LEG:-0}
i=0
for C in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d $OUT/${W}_$i -o run --output-format csv \
    -- python3 scripts/ab_dec.py --workload $W --legs $LEG --rounds 1 --iters 2 ${ARGS:-} \
    > $OUT/${W}_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/${W}_$i.log; exit 1; }
  echo "[pmc_ta] $W pass $i done"
done
