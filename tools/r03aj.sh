#!/bin/bash
# round-3 session aj: K6 with the glottal-tone filter fused into the output filter's loop
# (tonefused, tone_output_run) against the two runs back to back (tonek6); config 4 and config 3;
# then the tree GPU tests on tonefused
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03aj
AB="tonek6 tonefused" AB_PP=0 AB_SECONDS=0.5 bash tools/ab.sh || exit 3
AB="tonek6 tonefused" AB_PP=0 AB_ARGS="--workload vcv --batch 8192" bash tools/ab.sh 2>&1 | sed 's/^/vcv /'
AFS_LIB=$PWD/areafunctionsynthesis_amd/libafs_tonefused.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_target_sequence.py tests/test_adapter.py -x -v --timeout 300 --timeout-method thread -k "tree or target or adapter" > gpurun_out/r03aj/pytest.log 2>&1
st=$?; echo "pytest tonefused $st"; grep -A12 "parity report" gpurun_out/r03aj/pytest.log | cut -c1-230; tail -3 gpurun_out/r03aj/pytest.log
