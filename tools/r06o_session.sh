#!/bin/bash
# Round 6: hop-mode phase profile of the pair kernel p6 with the first phase group split finer.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06o
mkdir -p $OUT
export TMPDIR=/tmp
PP_HOPS=1 PP_PAIR_ROLES=1 PP_LIB=libphase_prof_p6.so timeout -k 10 240 python tools/phase_prof/run.py --batch 8192 --seconds 0.2 > $OUT/pp_p6_hops.txt 2>&1 || { cat $OUT/pp_p6_hops.txt; echo STOP pp p6; exit 3; }
cat $OUT/pp_p6_hops.txt
