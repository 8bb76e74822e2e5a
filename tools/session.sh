#!/bin/bash
# GPU session (run on the GPU box through gpurun): every step the rounds use, one script.
# Each GPU step runs under its own time limit; anything but pass / test failure (status 0 / 1)
# ends the script, so a fault, abort or timeout never starts another GPU step.
#
# usage: tools/session.sh TAG [steps...]      outputs under gpurun_out/TAG/
# steps (default: test smoke bench prof):
#   test    pytest -m gpu (PK="-k expression" narrows it)      smoke  __graft_entry__.smoke()
#   bench   bench.py $BENCH_ARGS                                prof   rocprofv3 --kernel-trace --stats of bench.py
#   pmc     FETCH_SIZE and WRITE_SIZE passes (one rocprofv3 run each) of one bench step
#   sq      SQ fp64 pass (tools/pmc_sq_fp64.py summarises it)  mix    three SQ instruction-mix passes
#   calib   the FETCH_SIZE calibration probe                    pp     per-phase cycle profile (tools/phase_prof)
#   ab      alternated A/B of in-tree variants (AB="tagA tagB", tools/ab.sh; built by tools/build_variant.sh)
# BENCH_ARGS: extra bench.py arguments for bench / prof / pmc / sq / mix (e.g. "--workload vcv").
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
STEPS=${*:-"test smoke bench prof"}
BA=${BENCH_ARGS:-}
ONE="--steps 1 --warmup 0 --no-cpu-baseline --no-sub-configs"
pmc() {  # pmc NAME "COUNTERS": one rocprofv3 counter pass over one bench step
  (cd /tmp && timeout -k 10 600 rocprofv3 --pmc $2 --kernel-trace --output-format csv -d $R/$OUT/$1 -o run -- python3 $R/bench.py $BA $ONE) > $OUT/$1.log 2>&1
  ok $? "$1"
}
for s in $STEPS; do
  case $s in
    test)  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PK:+-k "$PK"} > $OUT/pytest_gpu.log 2>&1; ok $? pytest
           grep -A14 "parity report" $OUT/pytest_gpu.log | cut -c1-240; tail -4 $OUT/pytest_gpu.log ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; ok $? smoke ;;
    bench) timeout -k 10 600 python bench.py $BA > $OUT/bench.json 2> $OUT/bench.err; ok $? bench; cat $OUT/bench.json ;;
    prof)  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py $BA --no-cpu-baseline --no-sub-configs) > $OUT/prof.log 2>&1; ok $? prof ;;
    pmc)   pmc pmc_fetch FETCH_SIZE; pmc pmc_write WRITE_SIZE ;;
    sq)    pmc pmc_sq "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FLOPS_FP64 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" ;;
    mix)   pmc pmc_mix1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64"
           pmc pmc_mix2 "SQ_WAVES SQ_INSTS_VALU_CVT SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
           pmc pmc_mix3 "SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY" ;;
    calib) (cd /tmp && timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/$OUT/calib -o run -- $R/tools/microbench/fetch_calib) > $OUT/calib.log 2>&1; ok $? calib ;;
    pp)    timeout -k 10 300 python tools/phase_prof/run.py --batch 8192 --seconds 0.02 > $OUT/phase_prof.txt 2>&1; ok $? phase_prof; cat $OUT/phase_prof.txt ;;
    ab)    timeout -k 10 1000 bash tools/ab.sh > $OUT/ab.txt 2>&1; ok $? ab; cat $OUT/ab.txt ;;
  esac
done
echo ALL DONE
