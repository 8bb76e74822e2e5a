#!/bin/bash
# Round 6: the wave-pair build (AFS_PAIR=1) against the default build: bitwise check of the audio at
# 16 lanes per utterance, then alternated timing (tools/ab.sh) at 8192 x 0.5 s and 65536 x 0.1 s.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06f
mkdir -p $OUT
export TMPDIR=/tmp
for t in base pair2; do
  AFS_EQ_LANES=16 AFS_LIB=$PWD/areafunctionsynthesis_amd/libafs_$t.so timeout -k 10 300 python tools/lib_equal.py write /tmp/eq_$t.npz > $OUT/eq_$t.log 2>&1 || { echo "eq $t failed ($?)"; tail -5 $OUT/eq_$t.log; exit 1; }
done
python tools/lib_equal.py compare /tmp/eq_base.npz /tmp/eq_pair2.npz | tee $OUT/eq_compare.txt
AB="base pair2 pair3" AB_BATCH=8192 AB_SECONDS=0.5 timeout -k 10 600 bash tools/ab.sh > $OUT/ab_8192.txt 2>&1; cat $OUT/ab_8192.txt
