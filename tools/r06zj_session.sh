#!/bin/bash
# Round 6: STAT priority always (pr3) against the default by batch (rounds of workgroups per CU slot:
# batch / 4096), 0.5 s utterances.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06zj
mkdir -p $OUT
export TMPDIR=/tmp
for b in 4096 8192 12288 16384 32768; do
  for t in cur pr3; do
    AFS_LIB=$PWD/areafunctionsynthesis_amd/libafs_$t.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-sub-configs --steps 2 --warmup 1 --seconds 0.5 --batch $b > $OUT/b${b}_$t.json 2> $OUT/b${b}_$t.err || { echo "STOP $b $t"; exit 3; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print('$t', $b, round(d['value']/1e6,2), 'M samples/s; K1', round(d['roofline']['avg_launch_ms'],1), 'ms')" $OUT/b${b}_$t.json
  done
done
