#!/bin/bash
# round-3 session o: K5 variants (pre-clamped LDS areas, loop unrolling): plan records against
# the host for each, then the 1 s bench alternated (K5 time per step)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03o
for t in prenu nu preu2; do
  AFS_LIB=$PWD/areafunctionsynthesis_amd/libafs_$t.so timeout -k 10 300 python -u -m pytest tests/test_plan_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r03o/plan_$t.log 2>&1
  st=$?; echo "plan tests $t: $st"; tail -1 gpurun_out/r03o/plan_$t.log
  if [ $st -ne 0 ] && [ $st -ne 1 ]; then exit $st; fi
done
AB="base prenu nu preu2" AB_PP=0 AB_SECONDS=1 bash tools/ab.sh || exit 3
