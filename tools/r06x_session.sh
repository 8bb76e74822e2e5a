#!/bin/bash
# Round 6: the pair kernel without the scheduling barriers at some phase marks: mA the noise phase's
# two, mB the first phase group's three, mC the solver's two -- alternated timing at 8192.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06x
mkdir -p $OUT
export TMPDIR=/tmp
AB="cur mA mB mC" AB_BATCH=8192 AB_SECONDS=0.5 timeout -k 10 700 bash tools/ab.sh > $OUT/ab_8192.txt 2>&1; cat $OUT/ab_8192.txt
