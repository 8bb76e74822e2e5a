#!/bin/bash
# Round 6: the slot order's keys retried with the wave-pair kernel (environment switches of the
# default build): class key first (1), XCD-dealt classes (3), no shape order; 8192 and 65536.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06r
mkdir -p $OUT
export TMPDIR=/tmp
AB="cur cur+AFS_CLASS_ORDER=1 cur+AFS_CLASS_ORDER=3 cur+AFS_SHAPE_ORDER=0 cur+AFS_NOISE_VARIANTS=2" AB_BATCH=8192 AB_SECONDS=0.5 timeout -k 10 700 bash tools/ab.sh > $OUT/ab_8192.txt 2>&1; cat $OUT/ab_8192.txt
AB="cur cur+AFS_CLASS_ORDER=1 cur+AFS_CLASS_ORDER=3" AB_BATCH=65536 AB_SECONDS=0.2 timeout -k 10 700 bash tools/ab.sh > $OUT/ab_65536.txt 2>&1; cat $OUT/ab_65536.txt
