#!/bin/bash
# round-3 session n: sequential K5 (default) vs K5 overlapped with K1 (AFS_PLAN_OVERLAP=1),
# 1 s steps, alternated three times
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03n
mkdir -p $OUT
for rep in 1 2 3; do
  for ov in 0 1; do
    AFS_PLAN_OVERLAP=$ov timeout -k 10 300 python bench.py --no-cpu-baseline --no-sub-configs --steps 2 --warmup 1 > $OUT/bench_ov${ov}_$rep.json 2> $OUT/bench_ov${ov}_$rep.err || { echo "STOP bench ov=$ov"; exit 3; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print('overlap=$ov', round(d['value']/1e6,2), 'M samples/s', round(d['ms_per_step'],1), 'ms/step', 'K1', round(d['roofline']['avg_launch_ms'],2), 'ms/launch', 'K5', round(d['roofline']['plan_kernel_ms_per_step'],1), 'ms/step')" $OUT/bench_ov${ov}_$rep.json
  done
done
