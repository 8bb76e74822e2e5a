#!/bin/bash
# Round 6: the pair kernel's lean solver with its record offsets in registers and the loads one
# (p5) or two (p4) positions ahead -- bitwise check, phase profiles, alternated timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06k
mkdir -p $OUT
export TMPDIR=/tmp
for t in p4 p5; do
  PP_PAIR_ROLES=1 PP_LIB=libphase_prof_$t.so timeout -k 10 240 python tools/phase_prof/run.py --batch 8192 --seconds 0.05 > $OUT/pp_$t.txt 2>&1 || { cat $OUT/pp_$t.txt; echo STOP pp $t; exit 3; }
  cat $OUT/pp_$t.txt
done
for t in base p4 p5; do
  AFS_EQ_LANES=16 AFS_LIB=$PWD/areafunctionsynthesis_amd/libafs_$t.so timeout -k 10 300 python tools/lib_equal.py write /tmp/eq_$t.npz > $OUT/eq_$t.log 2>&1 || { echo "eq $t failed ($?)"; tail -5 $OUT/eq_$t.log; exit 1; }
done
python tools/lib_equal.py compare /tmp/eq_base.npz /tmp/eq_p4.npz | tee $OUT/eq_compare.txt && python tools/lib_equal.py compare /tmp/eq_base.npz /tmp/eq_p5.npz | tee -a $OUT/eq_compare.txt
AB="base p3 p4 p5" AB_BATCH=8192 AB_SECONDS=0.5 timeout -k 10 600 bash tools/ab.sh > $OUT/ab_8192.txt 2>&1; cat $OUT/ab_8192.txt
