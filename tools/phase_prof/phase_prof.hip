// phase_prof.hip -- development tool: the tree kernel body with per-phase cycle counters
// (s_memtime deltas, accumulated per wave).  Not part of libafs; built by this directory's
// Makefile and driven by run.py on the GPU box.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "tree_kernel.h"

using namespace afs;
using namespace afs::tree;

// lanes per utterance of the profiled kernel (-DPP_W=64: the voice kernel)
#ifndef PP_W
#define PP_W TREE_W
#endif
constexpr int PW = PP_W;
constexpr int PWPB = Geom<PW>::WPB, PUPB = Geom<PW>::UPB;

__global__ void __launch_bounds__(64 * PWPB, AFS_TREE_MIN_WAVES) tree_prof_kernel(TreeArgs a, uint64_t *prof) {
  __shared__ WaveLdsT<PW> lds;
  tree_synth_body<true, AFS_GLOTTIS_TRIANGULAR, false, PW>(a, lds, prof);  // (the profiler runs the default glottis)
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return -1;                                                               \
    }                                                                          \
  } while (0)

extern "C" int pp_phase_count() { return PH_COUNT; }

// frames[B][F] host; cycles[PH_COUNT] = sum over waves; returns kernel ms in *ms.
static std::vector<uint64_t> g_wave;  // per-wave cycle totals of the last pp_run
extern "C" int pp_waves_per_block() { return PWPB; }
extern "C" void pp_wave_totals(uint64_t *out) {
  for (size_t w = 0; w < g_wave.size(); ++w) out[w] = g_wave[w];
}

extern "C" int pp_run(const afs_frame *frames, const uint32_t *seeds, int B, int F, int hop, double fs,
                      uint64_t *cycles, double *ms) {
  Tables *ht = new Tables();
  afs_options opt = afs::default_options();
  build_tables(ht, fs, opt);
  Tables *dt;
  afs_frame *df;
  uint32_t *ds;
  double *dout, *dlds;
  void *dlanes;
  uint64_t *dprof;
  double *dp25;  // section 25's pressures (K6's tone input; the kernel stores them every sample)
  const int blocks = (B + PUPB - 1) / PUPB, waves = blocks * PWPB;
  CK(hipMalloc(&dt, sizeof(Tables)));
  CK(hipMemcpy(dt, ht, sizeof(Tables), hipMemcpyHostToDevice));
  CK(hipMalloc(&df, sizeof(afs_frame) * B * F));
  CK(hipMemcpy(df, frames, sizeof(afs_frame) * B * F, hipMemcpyHostToDevice));
  CK(hipMalloc(&ds, 4 * B));
  CK(hipMemcpy(ds, seeds, 4 * B, hipMemcpyHostToDevice));
  CK(hipMalloc(&dout, sizeof(double) * (size_t)B * (F - 1) * hop));
  CK(hipMalloc(&dlds, sizeof(double) * (size_t)B * tree_lds_doubles()));
  CK(hipMalloc(&dlanes, (size_t)B * PW * tree_lane_bytes(PW)));
  CK(hipMalloc(&dprof, sizeof(uint64_t) * waves * PH_COUNT));
  CK(hipMalloc(&dp25, sizeof(double) * (size_t)B * (F - 1) * hop));
  CK(launch_tree_reset(dlanes, dlds, B, ds, PW, nullptr));
  const int64_t T = (int64_t)(F - 1) * hop;
  uint64_t *dplan;
  CK(hipMalloc(&dplan, (size_t)B * T * PLAN_RECORD_BYTES));
  PlanArgs pa{dt, df, F, B, hop, 0, T, dplan, T, 0, &dt->consts.sec[0]};
  CK(launch_plan(pa, nullptr));
  TreeArgs a{dt, df, F, nullptr, hop, 0, T, dout, T, dplan, T, dlanes, dlds, B, ht->uni, nullptr, 0, dp25, T};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, nullptr));
  hipLaunchKernelGGL(tree_prof_kernel, dim3(blocks), dim3(64 * PWPB), 0, nullptr, a, dprof);
  CK(hipGetLastError());
  CK(hipEventRecord(e1, nullptr));
  CK(hipEventSynchronize(e1));
  float fms = 0;
  CK(hipEventElapsedTime(&fms, e0, e1));
  *ms = fms;
  std::vector<uint64_t> h((size_t)waves * PH_COUNT);
  CK(hipMemcpy(h.data(), dprof, sizeof(uint64_t) * h.size(), hipMemcpyDeviceToHost));
  for (int p = 0; p < PH_COUNT; ++p) cycles[p] = 0;
  g_wave.assign(waves, 0);
  for (int w = 0; w < waves; ++w)
    for (int p = 0; p < PH_COUNT; ++p) {
      cycles[p] += h[(size_t)w * PH_COUNT + p];
      g_wave[w] += h[(size_t)w * PH_COUNT + p];
    }
  (void)hipFree(dt); (void)hipFree(df); (void)hipFree(ds); (void)hipFree(dout);
  (void)hipFree(dlds); (void)hipFree(dlanes); (void)hipFree(dprof); (void)hipFree(dplan); (void)hipFree(dp25);
  delete ht;
  return waves;
}
