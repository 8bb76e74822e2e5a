#!/bin/bash
# Round 6: a CU's second workgroup started ~half a sample (g1) or ~a whole sample (g2) after its
# first, against the default -- alternated timing at 8192 (two rounds) and 65536 (sixteen).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06w
mkdir -p $OUT
export TMPDIR=/tmp
AB="cur g1 g2" AB_BATCH=8192 AB_SECONDS=0.5 timeout -k 10 600 bash tools/ab.sh > $OUT/ab_8192.txt 2>&1; cat $OUT/ab_8192.txt
AB="cur g1" AB_BATCH=65536 AB_SECONDS=0.2 timeout -k 10 600 bash tools/ab.sh > $OUT/ab_65536.txt 2>&1; cat $OUT/ab_65536.txt
