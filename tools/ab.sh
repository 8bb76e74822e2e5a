#!/bin/bash
# A/B timing of kernel variants on the GPU box (development tool): for each tag T in $AB
# (default "A B"), the phase profile of tools/phase_prof/libphase_prof_T.so (AB_PP=1) and a short
# bench with areafunctionsynthesis_amd/libafs_T.so (AB_BATCH utterances, default 8192), alternating A B A B.  A tag "T+NAME=VALUE" runs
# variant T with the environment variable NAME=VALUE (e.g. "stage+AFS_PLAN_BUDGET_MB=48000").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for tag in ${AB:-A B}; do
    t=${tag%%+*}
    envs=""
    [ "$tag" != "$t" ] && envs=${tag#*+}
    if [ "${AB_PP:-0}" = 1 ]; then
      PP_LIB=libphase_prof_$t.so timeout -k 10 240 python tools/phase_prof/run.py --batch 8192 --seconds ${PP_SECONDS:-0.05} > gpurun_out/ab_pp_${t}_$rep.txt 2>&1 || { echo "STOP pp $t"; exit 3; }
      head -1 gpurun_out/ab_pp_${t}_$rep.txt; tail -1 gpurun_out/ab_pp_${t}_$rep.txt
    fi
    env $envs AFS_LIB=$PWD/areafunctionsynthesis_amd/libafs_$t.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-sub-configs --steps 2 --warmup 1 --seconds ${AB_SECONDS:-0.5} --batch ${AB_BATCH:-8192} ${AB_ARGS:-} > gpurun_out/ab_bench_${rep}_$tag.txt 2>&1 || { echo "STOP bench $tag"; exit 3; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print('$tag bench', round(d['value']/1e6,2), 'M samples/s', round(d['ms_per_step'],1), 'ms', 'launch', round(d['roofline']['avg_launch_ms'],2), 'x', d['roofline']['launches_per_step'], 'plan', round(d['roofline']['plan_kernel_ms_per_step'],2), 'K6', round(d['roofline']['output_kernel_ms_per_launch'],2))" gpurun_out/ab_bench_${rep}_$tag.txt
  done
done
