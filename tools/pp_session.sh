#!/bin/bash
# Development GPU session: tree-kernel parity subset + per-phase cycle profile.
# usage (on the GPU box): PP_K="tree" bash tools/pp_session.sh [tag]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-pp}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 -k "${PP_K:-tree}" > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP tests rc $rc"; exit $rc; fi
timeout -k 10 240 python tools/phase_prof/run.py --batch 8192 --seconds 0.02 > gpurun_out/${TAG}_prof.txt 2>&1 || { echo "STOP prof"; exit 3; }
cat gpurun_out/${TAG}_prof.txt
exit $rc
