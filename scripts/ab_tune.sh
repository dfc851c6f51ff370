#!/bin/bash
# Same-box A/B of tuning settings (and optionally an older build): scripts/ab_tune.sh <tag>
# <workloads> <setting>... ; a setting is "lib:<tag>" (FURY_ROW_LIB=fury_amd/libfury_row_<tag>.so)
# or "k=v,k2=v2" (fury_set_tuning).  3 interleaved rounds -> gpurun_out/ab_<tag>.jsonl
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; WL=$2; shift 2
OUT=gpurun_out/ab_$TAG.jsonl
mkdir -p gpurun_out; : > $OUT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for w in $WL; do
    for set in "$@"; do
      unset FURY_ROW_LIB
      tune="$set"
      case $set in lib:*) export FURY_ROW_LIB=$PWD/fury_amd/libfury_row_${set#lib:}.so; tune="";; esac
      timeout -k 10 240 python scripts/bench_tuned.py "$tune" --workload $w --steps 30 --warmup 5 \
        --no-cpu-baseline --no-e2e ${AB_EXTRA:-} > gpurun_out/ab_one.json 2> gpurun_out/ab_one.err
      rc=$?
      if [ $rc -ne 0 ]; then echo "bench $w $set rc=$rc"; tail -5 gpurun_out/ab_one.err; exit $rc; fi
      python - "$w" "$set" >> $OUT <<'PY'
import json, sys
d = json.load(open("gpurun_out/ab_one.json"))
r = d["roofline"]
print(json.dumps({"workload": sys.argv[1], "set": sys.argv[2], "value": d["value"],
                  "enc_ms": r["encode_ms"], "dec_ms": r["decode_ms"]}))
PY
      tail -1 $OUT
    done
  done
done
