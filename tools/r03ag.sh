#!/bin/bash
# round-3 session ag: the triangular glottis' two masses on the two halves of an utterance's lanes
# (split, -DAFS_GLOTTIS_SPLIT) against every lane evaluating both (nosplit); config 4 (two
# passes) and config 3; then the tree parity tests on the split build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03ag
AB="nosplit split" AB_PP=0 AB_SECONDS=0.5 bash tools/ab.sh || exit 3
AB="nosplit split" AB_PP=0 AB_SECONDS=0.5 bash tools/ab.sh || exit 3
AB="nosplit split" AB_PP=0 AB_ARGS="--workload vcv --batch 8192" bash tools/ab.sh 2>&1 | sed 's/^/vcv /'
AFS_LIB=$PWD/areafunctionsynthesis_amd/libafs_split.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_target_sequence.py tests/test_adapter.py -x -v --timeout 300 --timeout-method thread -k "tree or target or adapter" > gpurun_out/r03ag/pytest_split.log 2>&1
st=$?; echo "pytest split $st"; grep -A12 "parity report" gpurun_out/r03ag/pytest_split.log | cut -c1-250; tail -3 gpurun_out/r03ag/pytest_split.log
