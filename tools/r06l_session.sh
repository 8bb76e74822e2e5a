#!/bin/bash
# Round 6: phase profiles of the hop-mode kernels (K5's hop records, the noise-phase variants, slots
# ordered by noise class) for the default build and the wave-pair build p5, and both timed with the
# variants off (every wave the full noise phase).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06l
mkdir -p $OUT
export TMPDIR=/tmp
PP_HOPS=1 timeout -k 10 240 python tools/phase_prof/run.py --batch 8192 --seconds 0.2 > $OUT/pp_base_hops.txt 2>&1 || { cat $OUT/pp_base_hops.txt; echo STOP pp base; exit 3; }
cat $OUT/pp_base_hops.txt
PP_HOPS=1 PP_PAIR_ROLES=1 PP_LIB=libphase_prof_p5.so timeout -k 10 240 python tools/phase_prof/run.py --batch 8192 --seconds 0.2 > $OUT/pp_p5_hops.txt 2>&1 || { cat $OUT/pp_p5_hops.txt; echo STOP pp p5; exit 3; }
cat $OUT/pp_p5_hops.txt
AB="base+AFS_NOISE_VARIANTS=0 p5+AFS_NOISE_VARIANTS=0" AB_BATCH=8192 AB_SECONDS=0.5 timeout -k 10 600 bash tools/ab.sh > $OUT/ab_8192_full.txt 2>&1; cat $OUT/ab_8192_full.txt
