#!/bin/bash
# Round 6: the wave-pair kernel's rate against the batch (workgroup rounds per CU slot: 8192 -> 2,
# 16384 -> 4, 32768 -> 8, 65536 -> 16), 0.5 s utterances, default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06v
mkdir -p $OUT
export TMPDIR=/tmp
for b in 8192 12288 16384 24576 32768 65536; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-sub-configs --steps 2 --warmup 1 --seconds 0.5 --batch $b > $OUT/b$b.json 2> $OUT/b$b.err || { echo "STOP $b"; exit 3; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print($b, round(d['value']/1e6,2), 'M samples/s; K1', round(d['roofline']['avg_launch_ms'],1), 'ms')" $OUT/b$b.json
done
