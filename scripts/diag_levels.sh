#!/bin/bash
# DIAGNOSTIC: nested decode execute time with write phases switched off (FURY_LV_DBG bits, see
# levels.hip lv_dbg; outputs are wrong when a bit is set -- timing only), 4M depth-3 rows.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for d in 0 1 2 3 4 8 12; do
  FURY_DIAGNOSTIC=1 FURY_LV_DBG=$d timeout -k 10 300 python3 scripts/ab_generic.py --rows ${ROWS:-4000000} --iters 3 \
    > gpurun_out/diag_lv_$d.log 2>&1 || exit $?
  echo "dbg=$d $(tail -1 gpurun_out/diag_lv_$d.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["pieces_ms"])')"
done
