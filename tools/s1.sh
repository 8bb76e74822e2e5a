#!/bin/bash
# dev GPU session: tree parity subset, phase profile, short bench
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-s1}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "${PK:-tree or fricatives or af_to}" > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?
tail -25 gpurun_out/${TAG}_tests.txt
if [ $rc -ne 0 ]; then echo "STOP tests rc $rc"; exit $rc; fi
timeout -k 10 300 python tools/phase_prof/run.py --batch 8192 --seconds 0.02 > gpurun_out/${TAG}_prof.txt 2>&1 || { echo STOP prof; exit 3; }
cat gpurun_out/${TAG}_prof.txt
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo STOP bench; exit 4; }
cat gpurun_out/${TAG}_bench.json
