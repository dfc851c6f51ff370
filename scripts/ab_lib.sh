#!/bin/bash
# Same-box A/B of two builds of libfury_row (FURY_ROW_LIB = an older build kept in-tree as
# fury_amd/libfury_row_<tag>.so): the bench on each workload, builds interleaved, 3 rounds.
# Usage: scripts/ab_lib.sh <tag> [workloads...]   -> gpurun_out/ab_<tag>.jsonl
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
WL=${*:-struct100 mixed nested}
OUT=gpurun_out/ab_$TAG.jsonl
mkdir -p gpurun_out; : > $OUT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for w in $WL; do
    for lib in new old; do
      if [ $lib = old ]; then export FURY_ROW_LIB=$PWD/fury_amd/libfury_row_$TAG.so; else unset FURY_ROW_LIB; fi
      timeout -k 10 240 python bench.py --workload $w --steps 30 --warmup 5 --no-cpu-baseline --no-e2e > gpurun_out/ab_one.json 2> gpurun_out/ab_one.err
      rc=$?
      if [ $rc -ne 0 ]; then echo "bench $w $lib rc=$rc"; tail -5 gpurun_out/ab_one.err; exit $rc; fi
      python - "$w" "$lib" >> $OUT <<'PY'
import json, sys
d = json.load(open("gpurun_out/ab_one.json"))
r = d["roofline"]
print(json.dumps({"workload": sys.argv[1], "lib": sys.argv[2], "value": d["value"],
                  "enc_ms": r["encode_ms"], "dec_ms": r["decode_ms"]}))
PY
      tail -1 $OUT
    done
  done
done
