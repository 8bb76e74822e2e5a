#!/bin/bash
# round-3 session ab: state off the registers across the solver -- the radiation currents' old
# d/dt and smoothed flows read from LDS in the update (rad), and the dynamic sections' wall alpha
# through LDS / beta recomputed (radwall, default) -- against both in registers (regs); config 4
# and config 3; then the tree GPU tests on the default build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03ab
AB="regs rad radwall" AB_PP=0 AB_SECONDS=0.5 bash tools/ab.sh || exit 3
AB="regs radwall" AB_PP=0 AB_ARGS="--workload vcv --batch 8192" bash tools/ab.sh 2>&1 | sed 's/^/vcv /'
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_target_sequence.py tests/test_plan_gpu.py tests/test_adapter.py -x -v --timeout 300 --timeout-method thread -k "tree or target or plan_hops or adapter" > gpurun_out/r03ab/pytest.log 2>&1
st=$?; echo "pytest $st"; grep -A12 "parity report" gpurun_out/r03ab/pytest.log | cut -c1-250; tail -3 gpurun_out/r03ab/pytest.log
