#!/bin/bash
# round-4 session c: A/B of the output store windows (stage) against the single-lane stores
# (direct) and of one launch per step (plan budget 48 GB); phase profiles of both lane widths; SQ
# instruction mix, kernel trace and PMC traffic of HEAD; traffic of configs 5 and 3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04c; mkdir -p $OUT
AB="direct stage stage+AFS_PLAN_BUDGET_MB=48000" AB_SECONDS=1.0 bash tools/session.sh r04c ab || exit $?
timeout -k 10 300 python tools/phase_prof/run.py --batch 8192 --seconds 0.05 > $OUT/pp_w16.txt 2>&1 || { echo STOP pp16; exit 3; }
cat $OUT/pp_w16.txt
PP_LIB=libphase_prof_w64.so timeout -k 10 300 python tools/phase_prof/run.py --batch 1024 --seconds 0.05 > $OUT/pp_w64.txt 2>&1 || { echo STOP pp64; exit 3; }
cat $OUT/pp_w64.txt
bash tools/session.sh r04c mix prof || exit $?
BENCH_ARGS="--workload fricatives" bash tools/session.sh r04c_c5 pmc sq || exit $?
BENCH_ARGS="--workload vcv" bash tools/session.sh r04c_c3 pmc sq || exit $?
echo R04C DONE
