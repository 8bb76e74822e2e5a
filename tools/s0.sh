set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/phase_prof/run.py --batch 8192 --seconds 0.02 > gpurun_out/r02_base_prof.txt 2>&1 || { echo STOP prof; exit 3; }
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/r02_base_bench.json 2> gpurun_out/r02_base_bench.err || { echo STOP bench; exit 4; }
cat gpurun_out/r02_base_prof.txt gpurun_out/r02_base_bench.json
