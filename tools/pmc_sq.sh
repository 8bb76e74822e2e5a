#!/bin/bash
# SQ counter passes over the phase profiler's kernel (development tool; run on the GPU box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/pmc_sq
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${PP_ARGS:-"--batch 1024 --seconds 0.05"}
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY" \
           "SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_FLOPS_FP64" \
           "SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/phase_prof/run.py $ARGS) > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
