#!/bin/bash
# FETCH_SIZE calibration for gathered reads: tools/gather_probe's known-byte
# kernels under FETCH_SIZE and under the request-size counters, separate passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05_gather
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 tools/gather_probe > $OUT/plain.json 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- tools/gather_probe > $OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d $OUT/req -o run --output-format csv -- tools/gather_probe > $OUT/req.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum -d $OUT/dram -o run --output-format csv -- tools/gather_probe > $OUT/dram.log 2>&1 || exit 1
cat $OUT/plain.json
echo "[gather] done"
