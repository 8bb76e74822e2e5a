#!/bin/bash
# Round 6: K5 (tds_plan.hip) under the max-ilp (k5a) and iterative-ilp (k5b) schedulers against the
# default build -- alternated timing at 65536 x 0.2 s (K5's ms per step in the 'plan' column).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06ze
mkdir -p $OUT
export TMPDIR=/tmp
AB="cur k5a k5b" AB_BATCH=65536 AB_SECONDS=0.2 timeout -k 10 600 bash tools/ab.sh > $OUT/ab_65536.txt 2>&1; cat $OUT/ab_65536.txt
