#!/bin/bash
# round-3 session u: hop records (K5 hop mode) -- the plan / tree parity tests, then the bench
# alternated between hop records and dense records (AFS_PLAN_DENSE=1) on the same library
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_plan_gpu.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "${PK:-plan or tree or hop}" > $O/pytest.log 2>&1
st=$?; echo "pytest $st"; grep -A14 "parity report" $O/pytest.log | cut -c1-260; grep -E "PASS|FAIL|ERROR" $O/pytest.log | tail -40 | cut -c1-160; tail -3 $O/pytest.log
[ $st -gt 1 ] && exit 3
for rep in 1 2; do
  for mode in hops dense; do
    d=0; [ $mode = dense ] && d=1
    AFS_PLAN_DENSE=$d timeout -k 10 300 python bench.py --no-cpu-baseline --no-sub-configs --steps 2 --warmup 1 > $O/bench_${mode}_$rep.json 2> $O/bench_${mode}_$rep.err || { echo "STOP bench $mode"; exit 3; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); r=d['roofline']; print('$mode', round(d['value']/1e6,2), 'M samples/s', round(d['ms_per_step'],1), 'ms/step launch', round(r['avg_launch_ms'],2), 'plan ms/step', round(r.get('plan_kernel_ms_per_step',0),2))" $O/bench_${mode}_$rep.json
  done
done
