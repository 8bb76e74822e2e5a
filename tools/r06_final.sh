#!/bin/bash
# Round-6 measurement session (GPU box): tests, smoke, the bench line, its rocprof summary, the PMC
# traffic / SQ / instruction-mix passes of the 64k batch, the SQ pass of config 2 (voice kernel),
# phase profiles (the pair kernel by role, hop mode; the voice kernel).  Every GPU step has its own time limit; a fault, abort
# or timeout ends the script (tools/session.sh).  usage: tools/r06_final.sh TAG [steps]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:?tag}
shift
STEPS=${*:-"test bench prof pmc sq mix c2 pp"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for s in $STEPS; do
  case $s in
    test) bash tools/session.sh $TAG test smoke || exit $? ;;
    bench|prof|pmc|sq|mix) bash tools/session.sh $TAG $s || exit $? ;;
    c2) BENCH_ARGS="--batch 1024" bash tools/session.sh ${TAG}_c2 sq || exit $? ;;
    pp) PP_HOPS=1 PP_PAIR_ROLES=1 timeout -k 10 240 python tools/phase_prof/run.py --batch 65536 --seconds 0.02 > $OUT/pp_64k.txt 2>&1 || exit 1
        PP_PAIR_ROLES=1 PP_LIB=libphase_prof_w64.so timeout -k 10 200 python tools/phase_prof/run.py --batch 1024 --seconds 0.05 > $OUT/pp_w64_1024.txt 2>&1 || exit 1
        cat $OUT/pp_64k.txt $OUT/pp_w64_1024.txt ;;
    bal) timeout -k 10 300 python tools/shard_balance.py > $OUT/shard_balance.txt 2>&1 || exit 1; cat $OUT/shard_balance.txt ;;
  esac
done
echo FINAL DONE
