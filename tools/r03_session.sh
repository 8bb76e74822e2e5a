#!/bin/bash
# Round-3 GPU session (run on the GPU box): tests, smoke, bench, kernel-trace profile, PMC
# traffic passes (+ the FETCH_SIZE calibration probe) and the fp64 SQ pass.  Each GPU step has
# its own time limit; anything but pass / test failure ends the script.
# usage: tools/r03_session.sh TAG [steps...]   (steps: test smoke bench prof pmc sq calib avail mix pp spp)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:?tag}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
R=$PWD
ok() {
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP after $2 (status $1)"; exit "$1"; fi
  echo "$2 -> status $1"
}
STEPS=${*:-"test smoke bench prof pmc sq calib"}
BA=${BENCH_ARGS:-}
for s in $STEPS; do
  case $s in
    test)  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PK:+-k "$PK"} > $OUT/pytest_gpu.log 2>&1; ok $? pytest; tail -30 $OUT/pytest_gpu.log ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; ok $? smoke ;;
    bench) timeout -k 10 600 python bench.py $BA > $OUT/bench.json 2> $OUT/bench.err; ok $? bench; cat $OUT/bench.json ;;
    prof)  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py $BA --no-cpu-baseline --no-sub-configs) > $OUT/prof.log 2>&1; ok $? prof ;;
    pmc)   (cd /tmp && timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/$OUT/pmc_fetch -o run -- python3 $R/bench.py $BA --steps 1 --warmup 0 --no-cpu-baseline --no-sub-configs) > $OUT/pmc_fetch.log 2>&1; ok $? pmc_fetch
           (cd /tmp && timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/$OUT/pmc_write -o run -- python3 $R/bench.py $BA --steps 1 --warmup 0 --no-cpu-baseline --no-sub-configs) > $OUT/pmc_write.log 2>&1; ok $? pmc_write ;;
    sq)    (cd /tmp && timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FLOPS_FP64 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d $R/$OUT/pmc_sq -o run -- python3 $R/bench.py $BA --steps 1 --warmup 0 --no-cpu-baseline --no-sub-configs) > $OUT/pmc_sq.log 2>&1; ok $? pmc_sq ;;
    calib) (cd /tmp && timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/$OUT/calib -o run -- $R/tools/microbench/fetch_calib) > $OUT/calib.log 2>&1; ok $? calib ;;
    avail) (cd /tmp && timeout -k 10 120 rocprofv3 --list-avail) > $OUT/avail.txt 2>&1; ok $? avail ;;
    mix)   (cd /tmp && timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 --kernel-trace --output-format csv -d $R/$OUT/pmc_mix1 -o run -- python3 $R/bench.py $BA --steps 1 --warmup 0 --no-cpu-baseline --no-sub-configs) > $OUT/pmc_mix1.log 2>&1; ok $? pmc_mix1
           (cd /tmp && timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU_CVT SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-trace --output-format csv -d $R/$OUT/pmc_mix2 -o run -- python3 $R/bench.py $BA --steps 1 --warmup 0 --no-cpu-baseline --no-sub-configs) > $OUT/pmc_mix2.log 2>&1; ok $? pmc_mix2
           (cd /tmp && timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY --kernel-trace --output-format csv -d $R/$OUT/pmc_mix3 -o run -- python3 $R/bench.py $BA --steps 1 --warmup 0 --no-cpu-baseline --no-sub-configs) > $OUT/pmc_mix3.log 2>&1; ok $? pmc_mix3 ;;
    pp)    timeout -k 10 300 python tools/phase_prof/run.py --batch 8192 --seconds 0.02 > $OUT/phase_prof.txt 2>&1; ok $? phase_prof; cat $OUT/phase_prof.txt ;;
    spp)   timeout -k 10 300 python tools/phase_prof/seg_run.py --batch 8192 --seconds 0.02 > $OUT/seg_phase_prof.txt 2>&1; ok $? seg_phase_prof; cat $OUT/seg_phase_prof.txt ;;
  esac
done
echo ALL DONE
