#!/bin/bash
# Round 6: wave pairs with the rand() blocks on the DYN wave (pR) -- phase profile by role, A/B against
# the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06i
mkdir -p $OUT
export TMPDIR=/tmp
PP_PAIR_ROLES=1 PP_LIB=libphase_prof_pR.so timeout -k 10 240 python tools/phase_prof/run.py --batch 8192 --seconds 0.05 > $OUT/pp_pR.txt 2>&1 || { cat $OUT/pp_pR.txt; echo STOP pp; exit 3; }
cat $OUT/pp_pR.txt
timeout -k 10 240 python tools/phase_prof/run.py --batch 8192 --seconds 0.05 > $OUT/pp_base.txt 2>&1 || { echo STOP pp base; exit 3; }
cat $OUT/pp_base.txt
AB="base pR" AB_BATCH=8192 AB_SECONDS=0.5 timeout -k 10 600 bash tools/ab.sh > $OUT/ab_8192.txt 2>&1; cat $OUT/ab_8192.txt
