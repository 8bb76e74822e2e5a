#!/bin/bash
# Instruction-fetch counters over the phase profiler's kernel (development tool; GPU box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/pmc_if
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${PP_ARGS:-"--batch 1024 --seconds 0.05"}
(cd /tmp && timeout -k 10 300 rocprofv3 --pmc InstrFetchLatency --output-format csv -d $OUT/p2 -o run -- python3 $GRAFT_REPO_ROOT/tools/phase_prof/run.py $ARGS) > $OUT/p2.log 2>&1 || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ --output-format csv -d $OUT/p1 -o run -- python3 $GRAFT_REPO_ROOT/tools/phase_prof/run.py $ARGS) > $OUT/p1.log 2>&1 || exit 1
echo done
