#!/bin/bash
# Instruction-cache counters of a bench step for A/B library builds (development tool, GPU box):
# one rocprofv3 counter pass per tag T in $AB (areafunctionsynthesis_amd/libafs_T.so), each
# under its own time limit; summarised per kernel by tools/icache_summary.py.
# usage: tools/icache_probe.sh TAG       outputs under gpurun_out/TAG/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:?tag}
mkdir -p "$OUT"
export TMPDIR=/tmp
R=$PWD
for t in ${AB:-base nzvk}; do
  (cd /tmp && AFS_LIB=$R/areafunctionsynthesis_amd/libafs_$t.so timeout -s KILL 180 rocprofv3 \
     --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVES SQ_WAVE_CYCLES --kernel-trace --output-format csv \
     -d $R/$OUT/ic_$t -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-sub-configs \
     --seconds 0.5) > $OUT/ic_$t.log 2>&1 || { echo "STOP $t"; tail -5 $OUT/ic_$t.log; exit 3; }
  echo "$t done"
done
python3 tools/icache_summary.py $OUT ${AB:-base nzvk}
