#!/bin/bash
# Round 6: the shard's fixed per-launch time with the noise-phase variants off (every block the full
# phases: uniform block lengths) -- 8192 and 65536 utterances x 0.5 s, default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06zd
mkdir -p $OUT
export TMPDIR=/tmp
for v in 1 0; do
for b in 8192 65536; do
  AFS_NOISE_VARIANTS=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-sub-configs --steps 2 --warmup 1 --seconds 0.5 --batch $b > $OUT/b${b}_v$v.json 2> $OUT/b${b}_v$v.err || { echo "STOP $b"; exit 3; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print('variants $v', $b, round(d['value']/1e6,2), 'M samples/s; K1', round(d['roofline']['avg_launch_ms'],1), 'ms')" $OUT/b${b}_v$v.json
done
done
