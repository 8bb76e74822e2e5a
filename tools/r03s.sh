#!/bin/bash
# round-3 session s: one Newton step for the pivot / area reciprocals (rcp1), one row form for
# simple and bifurcation rows (rowu), both: A/B, then the tree solver's parity tests on "both"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03s
AB="base rcp1 rowu both" PP_SECONDS=0.05 AB_SECONDS=0.25 bash tools/ab.sh || exit 3
AFS_LIB=$PWD/areafunctionsynthesis_amd/libafs_both.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_target_sequence.py -x -v -k "tree or target" --timeout 300 --timeout-method thread > gpurun_out/r03s/pytest_both.log 2>&1
st=$?; echo "both pytest $st"; grep -A12 "parity report" gpurun_out/r03s/pytest_both.log | cut -c1-240; tail -2 gpurun_out/r03s/pytest_both.log
