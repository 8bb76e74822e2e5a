#!/bin/bash
# round-3 session ai: the glottal-tone filter in K6 from a stored p[25] per sample (tonek6,
# the default build since) against the filter inside the sample step (tonein, -DAFS_TONE_IN_KERNEL); config 4 and
# config 3; then the tree GPU tests on tonek6
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03ai
AB="tonein tonek6" AB_PP=0 AB_SECONDS=0.5 bash tools/ab.sh || exit 3
AB="tonein tonek6" AB_PP=0 AB_ARGS="--workload vcv --batch 8192" bash tools/ab.sh 2>&1 | sed 's/^/vcv /'
AFS_LIB=$PWD/areafunctionsynthesis_amd/libafs_tonek6.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_target_sequence.py tests/test_adapter.py -x -v --timeout 300 --timeout-method thread -k "tree or target or adapter" > gpurun_out/r03ai/pytest.log 2>&1
st=$?; echo "pytest tonek6 $st"; grep -A12 "parity report" gpurun_out/r03ai/pytest.log | cut -c1-230; tail -3 gpurun_out/r03ai/pytest.log
