#!/bin/bash
# Round 6: the grouped row walk at its defaults -- A/B vs the level engine, rocprof kernel stats of
# the 128-counted-node decode -- then the nested / fuzz / bounds tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R06_OUT:-r06g4}
mkdir -p $OUT
export TMPDIR=/tmp
R06_OUT=$R06_OUT SWEEP="walk_group_k=4" GLEGS="[{}]" PROF=1 bash scripts/r06_group2.sh || exit 1
timeout -k 10 300 python -u scripts/ab_deep.py --levels "" --wide 64,128,200 --rows 1000000 --modes 2,1 > $OUT/ab_default.log 2>&1 || { tail -20 $OUT/ab_default.log; exit 1; }
grep "^{" $OUT/ab_default.log
R06_OUT=$R06_OUT GKS=" " LEGS_RUN=0 TESTS=1 bash scripts/r06_group.sh
