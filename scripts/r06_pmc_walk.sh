#!/bin/bash
# Round 6: row-walk decode traffic (separate --pmc passes, no tracing): the 4M depth-3 batch at the
# defaults (one group) and the 1M-row bean of 128 counted nodes (field groups of 4).  WRITE_SIZE
# and the read requests (x 128 B: every gfx950 fabric read is a 128-B line, r05_gather_probe).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${PMC_OUT:-r06_pmc_walk}
mkdir -p $OUT
export TMPDIR=/tmp
run() {   # name, then the program
  local n=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $OUT/$n/w -o run --output-format csv -- "$@" > $OUT/$n.w.log 2>&1 || { tail -5 $OUT/$n.w.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum -d $OUT/$n/r -o run --output-format csv -- "$@" > $OUT/$n.r.log 2>&1 || { tail -5 $OUT/$n.r.log; exit 1; }
  echo "[pmc] $n done"
}
run depth3 python3 scripts/ab_generic.py --rows 4000000 --iters 1 --legs '[{}]'
run counted128 python3 scripts/ab_deep.py --levels "" --wide 128 --rows 1000000 --modes 2 --iters 1
