#!/bin/bash
# Round 6: the pair kernel's STAT wave without the glottis evaluation (s2: DYN commits it, STAT
# evaluates the upper area alone) -- bitwise check against the one-wave build, alternated timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06s
mkdir -p $OUT
export TMPDIR=/tmp
for t in base s2; do
  AFS_EQ_LANES=16 AFS_LIB=$PWD/areafunctionsynthesis_amd/libafs_$t.so timeout -k 10 300 python tools/lib_equal.py write /tmp/eq_$t.npz > $OUT/eq_$t.log 2>&1 || { echo "eq $t failed ($?)"; tail -5 $OUT/eq_$t.log; exit 1; }
done
python tools/lib_equal.py compare /tmp/eq_base.npz /tmp/eq_s2.npz | tee $OUT/eq_compare.txt
AB="cur s2" AB_BATCH=8192 AB_SECONDS=0.5 timeout -k 10 600 bash tools/ab.sh > $OUT/ab_8192.txt 2>&1; cat $OUT/ab_8192.txt
AB="cur s2" AB_BATCH=65536 AB_SECONDS=0.2 timeout -k 10 600 bash tools/ab.sh > $OUT/ab_65536.txt 2>&1; cat $OUT/ab_65536.txt
