#!/bin/bash
# Round 6 (diagnostic, wrong audio by design): the pair kernel with the STAT wave's solver skipped
# (qNS) or its targets + noise skipped (qNN) -- how much of each the sample's time is.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06zf
mkdir -p $OUT
export TMPDIR=/tmp
AB="cur qNS qNN" AB_BATCH=8192 AB_SECONDS=0.5 timeout -k 10 600 bash tools/ab.sh > $OUT/ab_8192.txt 2>&1; cat $OUT/ab_8192.txt
