#!/bin/bash
# Round 6: the pair kernel with a scheduling barrier at every phase mark (p6) against the default
# build and p5 -- bitwise check, hop-mode phase profile, alternated timing (variants on and off).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06m
mkdir -p $OUT
export TMPDIR=/tmp
for t in base p6; do
  AFS_EQ_LANES=16 AFS_LIB=$PWD/areafunctionsynthesis_amd/libafs_$t.so timeout -k 10 300 python tools/lib_equal.py write /tmp/eq_$t.npz > $OUT/eq_$t.log 2>&1 || { echo "eq $t failed ($?)"; tail -5 $OUT/eq_$t.log; exit 1; }
done
python tools/lib_equal.py compare /tmp/eq_base.npz /tmp/eq_p6.npz | tee $OUT/eq_compare.txt
AB="base p5 p6 p6+AFS_NOISE_VARIANTS=0" AB_BATCH=8192 AB_SECONDS=0.5 timeout -k 10 600 bash tools/ab.sh > $OUT/ab_8192.txt 2>&1; cat $OUT/ab_8192.txt
