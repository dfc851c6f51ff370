#!/bin/bash
# Row-walk decode traffic at 4M depth-3 rows under tuning legs (LEGS: JSON objects of tuning keys,
# one per leg, ';'-separated): WRITE_SIZE, and the read-request counters (every fabric read is a
# 128-B line on gfx950: scripts/r05_gather_probe.sh).  Separate --pmc passes, no tracing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${PMC_OUT:-r05_pmc_walk}
mkdir -p $OUT
export TMPDIR=/tmp
IFS=';' read -ra LEGA <<< "${LEGS:-{\"walk_out\":0};{\"walk_out\":16384}}"
i=0
for L in "${LEGA[@]}"; do
  i=$((i+1))
  echo "$L" > $OUT/leg$i.txt
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $OUT/w$i -o run --output-format csv -- python3 scripts/ab_generic.py --rows 4000000 --iters 1 --legs "[$L]" > $OUT/w$i.log 2>&1 || exit 1
  if [ "${READS:-1}" = "1" ]; then
    timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum -d $OUT/r$i -o run --output-format csv -- python3 scripts/ab_generic.py --rows 4000000 --iters 1 --legs "[$L]" > $OUT/r$i.log 2>&1 || exit 1
  fi
  echo "[pmc_walk] leg $i $L done"
done
