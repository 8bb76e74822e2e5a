#!/bin/bash
# Round 6: wave pairs placed by SIMD (AFS_PAIR_MAP 3: each SIMD one DYN and one STAT wave of its CU's
# two workgroups) -- bitwise check against the default build, phase profiles with the placement
# analysis (map 0 and map 3), alternated timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06j
mkdir -p $OUT
export TMPDIR=/tmp
for t in pR p3; do
  PP_PAIR_ROLES=1 PP_LIB=libphase_prof_$t.so timeout -k 10 240 python tools/phase_prof/run.py --batch 8192 --seconds 0.05 > $OUT/pp_$t.txt 2>&1 || { cat $OUT/pp_$t.txt; echo STOP pp $t; exit 3; }
  cat $OUT/pp_$t.txt
done
for t in base p3; do
  AFS_EQ_LANES=16 AFS_LIB=$PWD/areafunctionsynthesis_amd/libafs_$t.so timeout -k 10 300 python tools/lib_equal.py write /tmp/eq_$t.npz > $OUT/eq_$t.log 2>&1 || { echo "eq $t failed ($?)"; tail -5 $OUT/eq_$t.log; exit 1; }
done
python tools/lib_equal.py compare /tmp/eq_base.npz /tmp/eq_p3.npz | tee $OUT/eq_compare.txt
AB="base pR p3" AB_BATCH=8192 AB_SECONDS=0.5 timeout -k 10 600 bash tools/ab.sh > $OUT/ab_8192.txt 2>&1; cat $OUT/ab_8192.txt
