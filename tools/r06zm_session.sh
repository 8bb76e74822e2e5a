#!/bin/bash
# Round 6: the STAT priority modes at run time (AFS_STAT_PRIO; new = the build with the modes, default
# 2 at >= 2 rounds) -- 4096 (one round), 16384 (four), 65536 (sixteen; cur = the previous default).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06zm
mkdir -p $OUT
export TMPDIR=/tmp
AB="new+AFS_STAT_PRIO=0 new+AFS_STAT_PRIO=2 new+AFS_STAT_PRIO=3" AB_BATCH=4096 AB_SECONDS=0.5 timeout -k 10 600 bash tools/ab.sh > $OUT/ab_4096.txt 2>&1; cat $OUT/ab_4096.txt
AB="new+AFS_STAT_PRIO=0 new new+AFS_STAT_PRIO=3" AB_BATCH=16384 AB_SECONDS=0.5 timeout -k 10 600 bash tools/ab.sh > $OUT/ab_16384.txt 2>&1; cat $OUT/ab_16384.txt
AB="cur new" AB_BATCH=65536 AB_SECONDS=0.2 timeout -k 10 600 bash tools/ab.sh > $OUT/ab_65536.txt 2>&1; cat $OUT/ab_65536.txt
