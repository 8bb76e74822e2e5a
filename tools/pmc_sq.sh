#!/bin/bash
# SQ counter passes over the phase profiler's kernel (development tool; run on the GPU box).
# One rocprofv3 run per pass (at most 8 SQ counters each); summary by tools/pmc_sq_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/pmc_sq
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${PP_ARGS:-"--batch 8192 --seconds 0.02"}
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FLOPS_FP64" \
           "SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU2 SQ_INSTS_VSKIPPED SQ_IFETCH SQ_INSTS_SMEM SQ_THREAD_CYCLES_VALU"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/phase_prof/run.py $ARGS) > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
