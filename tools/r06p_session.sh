#!/bin/bash
# Round 6: the pair kernel with the first phase group split (p9: DYN evaluates the glottis alone)
# against p6 and the default build -- bitwise check, hop-mode phase profile, alternated timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06p
mkdir -p $OUT
export TMPDIR=/tmp
for t in base p9; do
  AFS_EQ_LANES=16 AFS_LIB=$PWD/areafunctionsynthesis_amd/libafs_$t.so timeout -k 10 300 python tools/lib_equal.py write /tmp/eq_$t.npz > $OUT/eq_$t.log 2>&1 || { echo "eq $t failed ($?)"; tail -5 $OUT/eq_$t.log; exit 1; }
done
python tools/lib_equal.py compare /tmp/eq_base.npz /tmp/eq_p9.npz | tee $OUT/eq_compare.txt
PP_HOPS=1 PP_PAIR_ROLES=1 PP_LIB=libphase_prof_p9.so timeout -k 10 240 python tools/phase_prof/run.py --batch 8192 --seconds 0.2 > $OUT/pp_p9_hops.txt 2>&1 || { cat $OUT/pp_p9_hops.txt; echo STOP pp p9; exit 3; }
cat $OUT/pp_p9_hops.txt
AB="base p6 p9" AB_BATCH=8192 AB_SECONDS=0.5 timeout -k 10 600 bash tools/ab.sh > $OUT/ab_8192.txt 2>&1; cat $OUT/ab_8192.txt
