#!/bin/bash
# Round 6: the pair kernel under other machine schedulers (sA max-ilp, sB iterative-minreg) and with
# the rand() blocks back on the STAT wave (sC), against the default -- alternated timing at 8192.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06u
mkdir -p $OUT
export TMPDIR=/tmp
AB="cur sA sB sC" AB_BATCH=8192 AB_SECONDS=0.5 timeout -k 10 700 bash tools/ab.sh > $OUT/ab_8192.txt 2>&1; cat $OUT/ab_8192.txt
