#!/bin/bash
# Round 6: STAT priority always (pr3) against the default at 65536 x 0.2 s, config 2 (1024 x 0.5 s,
# the voice pairs) and one voice (latency).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06zi
mkdir -p $OUT
export TMPDIR=/tmp
AB="cur pr3" AB_BATCH=65536 AB_SECONDS=0.2 timeout -k 10 600 bash tools/ab.sh > $OUT/ab_65536.txt 2>&1; cat $OUT/ab_65536.txt
AB="cur pr3" AB_BATCH=1024 AB_SECONDS=0.5 timeout -k 10 600 bash tools/ab.sh > $OUT/ab_1024.txt 2>&1; cat $OUT/ab_1024.txt
AB="cur pr3" AB_BATCH=1 AB_SECONDS=0.5 timeout -k 10 600 bash tools/ab.sh > $OUT/ab_1.txt 2>&1; cat $OUT/ab_1.txt
