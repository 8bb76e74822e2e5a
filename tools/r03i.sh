#!/bin/bash
# round-3 session i: K5 plan records of the new K5 against the host, then A/B (1 s steps) of
# the previous build (base), K1 issue priority over the overlapped K5 (prio), the cheaper K5 (k5).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03i
timeout -k 10 400 python -u -m pytest tests/test_plan_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03i/plan.log 2>&1
st=$?; echo "plan tests $st"; tail -2 gpurun_out/r03i/plan.log
if [ $st -ne 0 ] && [ $st -ne 1 ]; then exit $st; fi
AB="base prio k5" AB_PP=0 AB_SECONDS=1 bash tools/ab.sh || exit 3
