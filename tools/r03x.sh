#!/bin/bash
# round-3 session x: the output stage as its own kernel K6 (k6, the default build) against the
# output filter inside the synthesis kernel (base: -DAFS_K1_FILTER -DAFS_CLAMP_TWICE = HEAD) and
# K6 without the single area clamp per slot (k6c2); config 4 and config 3; then the tree GPU
# tests on the default build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03x
AB="base k6 k6c2" AB_PP=0 AB_SECONDS=0.5 bash tools/ab.sh || exit 3
AB="base k6" AB_PP=0 AB_ARGS="--workload vcv --batch 8192" bash tools/ab.sh 2>&1 | sed 's/^/vcv /' || exit 3
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_target_sequence.py tests/test_adapter.py tests/test_plan_gpu.py -x -v --timeout 300 --timeout-method thread -k "tree or target or adapter or session or plan_hops" > gpurun_out/r03x/pytest.log 2>&1
st=$?; echo "pytest $st"; grep -A12 "parity report" gpurun_out/r03x/pytest.log | cut -c1-250; tail -3 gpurun_out/r03x/pytest.log
