#!/bin/bash
# Round 6: priority modes 4 / 5 (mode 2 plus the DYN wave's rows at priority 2 / 1) against mode 2 (the
# default) -- alternated timing at 8192 x 0.5 s and 65536 x 0.2 s.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06zo
mkdir -p $OUT
export TMPDIR=/tmp
AB="new new+AFS_STAT_PRIO=4 new+AFS_STAT_PRIO=5" AB_BATCH=8192 AB_SECONDS=0.5 timeout -k 10 600 bash tools/ab.sh > $OUT/ab_8192.txt 2>&1; cat $OUT/ab_8192.txt
AB="new new+AFS_STAT_PRIO=4 new+AFS_STAT_PRIO=5" AB_BATCH=65536 AB_SECONDS=0.2 timeout -k 10 600 bash tools/ab.sh > $OUT/ab_65536.txt 2>&1; cat $OUT/ab_65536.txt
