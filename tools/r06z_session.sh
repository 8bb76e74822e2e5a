#!/bin/bash
# Round 6: the voice kernel as wave pairs (tree_pair64_kernel, batches <= 512) -- bitwise check at 64
# lanes against the one-wave build, the real-time test, small-batch rates.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06z
mkdir -p $OUT
export TMPDIR=/tmp
for t in base cur; do
  AFS_EQ_LANES=64 AFS_LIB=$PWD/areafunctionsynthesis_amd/libafs_$t.so timeout -k 10 300 python tools/lib_equal.py write /tmp/eq_$t.npz > $OUT/eq_$t.log 2>&1 || { echo "eq $t failed ($?)"; tail -5 $OUT/eq_$t.log; exit 1; }
done
python tools/lib_equal.py compare /tmp/eq_base.npz /tmp/eq_cur.npz | tee $OUT/eq_compare.txt
timeout -k 10 300 python -u -m pytest tests/test_adapter.py -x -v --timeout 200 --timeout-method thread -k "real" -s > $OUT/rt.log 2>&1; echo "rt status $?"; grep -E "wall time|passed|failed" $OUT/rt.log | cut -c1-300
for b in 1 64 512 1024; do
  for t in base cur; do
    AFS_LIB=$PWD/areafunctionsynthesis_amd/libafs_$t.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-sub-configs --steps 2 --warmup 1 --seconds 0.5 --batch $b > $OUT/b${b}_$t.json 2> $OUT/b${b}_$t.err || { echo "STOP $b $t"; tail -3 $OUT/b${b}_$t.err; exit 3; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print('$t', $b, round(d['value']/1e6,3), 'M samples/s; K1', round(d['roofline']['avg_launch_ms'],2), 'ms', d['roofline']['kernel'])" $OUT/b${b}_$t.json
  done
done
