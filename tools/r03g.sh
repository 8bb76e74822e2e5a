#!/bin/bash
# round-3 session g: the -disable-machine-cse reproducer, the counter list, A/B of the tree
# kernel built with -disable-machine-cse, and its tree parity tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03g
mkdir -p $OUT
timeout -k 10 60 tools/microbench/cse_default > $OUT/cse_default.txt 2>&1; echo "repro default $?"; cat $OUT/cse_default.txt
timeout -k 10 60 tools/microbench/cse_off > $OUT/cse_off.txt 2>&1; echo "repro cse-off $?"; cat $OUT/cse_off.txt
(cd /tmp && timeout -k 10 120 rocprofv3 --list-avail) > $OUT/avail.txt 2>&1; echo "avail $?"
AB="base treecse" bash tools/ab.sh || exit 3
AFS_LIB=$PWD/areafunctionsynthesis_amd/libafs_treecse.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v -k "tree" --timeout 300 --timeout-method thread > $OUT/treecse_pytest.log 2>&1
st=$?; echo "treecse pytest $st"; tail -12 $OUT/treecse_pytest.log
