#!/bin/bash
# Run on the GPU box: tests, smoke, bench, profile.  Each GPU step has its own time
# limit; a crash/timeout (anything but pass/test-failure) ends the script.
# usage: tools/gpu_session.sh [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
ok() { # $1=status $2=step ; pytest 1 = test failures (no fault): continue
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP after $2 (status $1)"; exit "$1"; fi
  echo "$2 -> status $1"
}
STEPS=${STEPS:-"test smoke bench prof"}
for s in $STEPS; do
  case $s in
    test)  timeout -k 10 900 python -m pytest tests -m gpu -q -x > $OUT/pytest_gpu.log 2>&1; ok $? pytest ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; ok $? smoke ;;
    bench) timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1; ok $? bench ;;
    prof)  (cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py ${BENCH_ARGS:-} --no-cpu-baseline) > $OUT/prof.log 2>&1; ok $? prof ;;
    pmc)   (cd /tmp && timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/pmc_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py ${BENCH_ARGS:-} --no-cpu-baseline) > $OUT/pmc_fetch.log 2>&1; ok $? pmc_fetch
           (cd /tmp && timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/pmc_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py ${BENCH_ARGS:-} --no-cpu-baseline) > $OUT/pmc_write.log 2>&1; ok $? pmc_write ;;
  esac
done
echo ALL DONE
