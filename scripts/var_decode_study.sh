#!/bin/bash
# Round-2 study of the variable-length decode: the default register-staged kernel
# vs the LDS-staged one (var_decode = 4) under diagnostic legs -- ticket vs blockIdx order (4096),
# no look-back (32), staging only (128), no payload (16), no fixed stores (8) -- and tile sizes.
# One JSON line per run into gpurun_out/var_decode_study.jsonl.  Every step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/var_decode_study.jsonl
mkdir -p gpurun_out
: > $OUT
run() {   # env-assignments... -- args
  timeout -k 10 200 env "$@" python -u scripts/time_decode.py ${LEGS} 2>/dev/null | tail -1 >> $OUT || exit 1
}
LEGS="--legs 0:0,0:128,0:4096,0:32,3:0,3:128,4:0,4:4096,4:4128,4:4224,4:4112,4:4104"
run FURY_LDS_ROWS=256
LEGS="--legs 4:4096,4:4128,4:4224"
run FURY_LDS_ROWS=128 FURY_LDS_BUDGET=30000
LEGS="--workload nested --legs 0:0,0:128,3:0,4:0,4:4096"
run FURY_LDS_ROWS=256
cat $OUT
