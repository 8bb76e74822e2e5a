#!/bin/bash
# round-3 session y: the next frame loaded a sample ahead in the dense kernel (pf, default) against
# frame_load at each transition (nopf), config 3 (hop 1) and config 4; then the full GPU suite
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03y
AB="nopf pf" AB_PP=0 AB_ARGS="--workload vcv --batch 8192" bash tools/ab.sh 2>&1 | sed 's/^/vcv /'
AB="nopf pf" AB_PP=0 AB_SECONDS=0.5 bash tools/ab.sh || exit 3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03y/pytest.log 2>&1
st=$?; echo "pytest $st"; grep -A16 "parity report" gpurun_out/r03y/pytest.log | cut -c1-250; tail -3 gpurun_out/r03y/pytest.log
