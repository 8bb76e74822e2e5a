#!/bin/bash
# A/B builds (development tool): libafs_TAG.so and libphase_prof_TAG.so from the current tree
# with extra compiler flags (e.g. -DAFS_VAR_...), for tools/ab.sh.
# usage: tools/build_variant.sh TAG "FLAGS"
set -eu
cd "$(dirname "$0")/.."
TAG=$1
FLAGS=${2:-}
C=areafunctionsynthesis_amd/csrc
O=/tmp/afs_variant_$TAG
mkdir -p $O
# the tree kernel's flags as build.py TREE_FLAGS (TREE_BASE overrides them, TREE_EXTRA adds)
TREE_BASE=${TREE_BASE:-"-mllvm -disable-machine-licm -ffp-contract=fast-honor-pragmas -fno-signed-zeros -mllvm -amdgpu-sched-strategy=iterative-ilp"}
COMMON="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function -ffp-contract=off -fno-strict-aliasing -Wno-unknown-pragmas --offload-arch=gfx950 $FLAGS"
objs=""
for s in afs_capi.cpp afs_comm.cpp afs_tables.cpp tds_lane.hip tds_tree.hip tds_plan.hip af_kernels.hip audio_kernels.hip; do
  o=$O/${s%.*}.o
  extra=""
  [ $s = tds_tree.hip ] && extra="$TREE_BASE ${TREE_EXTRA:-}"  # (as build.py)
  [ $s = tds_plan.hip ] && extra="${PLAN_EXTRA:-}"
  /opt/rocm/bin/hipcc -c -x hip $C/$s -o $o $COMMON $extra &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc -shared -o areafunctionsynthesis_amd/libafs_$TAG.so --offload-arch=gfx950 -fPIC $objs -ldl
/opt/rocm/bin/hipcc -shared -o tools/phase_prof/libphase_prof_$TAG.so $COMMON $TREE_BASE -I$C -Iinclude ${TREE_EXTRA:-} tools/phase_prof/phase_prof.hip -x hip $C/afs_tables.cpp $C/tds_tree.hip $C/tds_plan.hip
echo built $TAG
