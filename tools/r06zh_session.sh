#!/bin/bash
# Round 6: the STAT wave's issue priority over its SIMD's DYN wave (s_setprio 2): during the solver
# (pr1), the first phase group and the solver (pr2), always (pr3) -- alternated timing at 8192.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06zh
mkdir -p $OUT
export TMPDIR=/tmp
AB="cur pr1 pr2 pr3" AB_BATCH=8192 AB_SECONDS=0.5 timeout -k 10 700 bash tools/ab.sh > $OUT/ab_8192.txt 2>&1; cat $OUT/ab_8192.txt
