#!/bin/bash
# Round 6: wave-pair placement / scheduler variants against the default build (alternated, tools/ab.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06h
mkdir -p $OUT
export TMPDIR=/tmp
AB="${AB_LIST:-base pA pC pair}" AB_BATCH=8192 AB_SECONDS=0.5 timeout -k 10 900 bash tools/ab.sh > $OUT/ab_8192.txt 2>&1; cat $OUT/ab_8192.txt
