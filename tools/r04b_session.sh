set -u
cd $GRAFT_REPO_ROOT
bash tools/session.sh r04b test smoke bench pmc || exit $?
for L in 16 64; do
  timeout -k 10 300 python bench.py --batch 1024 --lanes $L --steps 2 --warmup 1 --no-cpu-baseline --no-sub-configs > gpurun_out/r04b/bench_c2_L$L.json 2> gpurun_out/r04b/bench_c2_L$L.err || { echo "STOP c2 $L"; exit 3; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print('config2 lanes $L', round(d['value']/1e6,2), 'M samples/s', round(d['roofline']['avg_launch_ms'],2), 'ms/launch')" gpurun_out/r04b/bench_c2_L$L.json
done
