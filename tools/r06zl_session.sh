#!/bin/bash
# Round 6: STAT priority during the solver (pr1) or the first group + the solver (pr2) at 65536 x 0.2 s
# against the default (no priority at 16 rounds).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06zl
mkdir -p $OUT
export TMPDIR=/tmp
AB="cur pr1 pr2" AB_BATCH=65536 AB_SECONDS=0.2 timeout -k 10 600 bash tools/ab.sh > $OUT/ab_65536.txt 2>&1; cat $OUT/ab_65536.txt
