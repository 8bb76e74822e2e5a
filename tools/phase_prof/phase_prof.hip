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
#define PP_W AFS_TREE_W
#endif
constexpr int PW = PP_W;
// (HOPS: K5's hop records and the noise-phase variants, as the library's large calls run)
#if AFS_PAIR && PP_W == AFS_TREE_W
// the wave-pair kernel (AFS_PAIR=1 builds, 16 lanes per utterance): four waves per block
constexpr int PWPB = 4, PUPB = Geom<PW>::UPB;
template <bool HOPS>
__global__ void __launch_bounds__(256, 2) tree_prof_kernel(TreeArgs a, uint64_t *prof) {
  __shared__ WaveLdsT<TW> lds;
  __shared__ int pattern[5];
  tree_pair_body<AFS_GLOTTIS_TRIANGULAR, HOPS, true>(a, lds, pattern, prof);
}
#elif AFS_PAIR && PP_W == 64
// the voice kernel's pairs (AFS_PAIR builds, -DPP_W=64): two waves per utterance
constexpr int PWPB = 2, PUPB = 1;
template <bool HOPS>
__global__ void __launch_bounds__(128, AFS_PAIR64_WAVES) tree_prof_kernel(TreeArgs a, uint64_t *prof) {
  __shared__ WaveLdsT<64> lds;
  tree_pair64_body<AFS_GLOTTIS_TRIANGULAR, HOPS, true>(a, lds, prof);
}
#else
constexpr int PWPB = Geom<PW>::WPB, PUPB = Geom<PW>::UPB;

template <bool HOPS>
__global__ void __launch_bounds__(64 * PWPB, AFS_TREE_MIN_WAVES) tree_prof_kernel(TreeArgs a, uint64_t *prof) {
  __shared__ WaveLdsT<PW> lds;
  tree_synth_body<true, AFS_GLOTTIS_TRIANGULAR, HOPS, PW>(a, lds, prof);  // (the profiler runs the default glottis)
}
#endif
static int g_hops = 0;
extern "C" void pp_set_hops(int on) { g_hops = on; }

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
static std::vector<uint64_t> g_wave_ph;  // per-wave, per-phase cycles of the last pp_run
extern "C" void pp_wave_phases(uint64_t *out) {
  for (size_t w = 0; w < g_wave_ph.size(); ++w) out[w] = g_wave_ph[w];
}
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
  PlanHop *dhops = nullptr;
  uint32_t *dwork = nullptr;
  int32_t *dorder = nullptr;
  const int64_t hstride = plan_hop_slots(0, T, hop);
  CK(hipMalloc(&dplan, (size_t)B * (g_hops ? hstride * hop : T) * PLAN_RECORD_BYTES));
  TreeArgs a{dt, df, F, nullptr, hop, 0, T, dout, T, dplan, T, dlanes, dlds, B, ht->uni, nullptr, 0, dp25, T};
  if (!g_hops) {
    PlanArgs pa{dt, df, F, B, hop, 0, T, dplan, T, 0, &dt->consts.sec[0]};
    CK(launch_plan(pa, nullptr));
  } else {
    // hop records, every mixed hop a compact slot; the slots ordered by noise class as the library's
    // slot order keys them (afs_capi.cpp shape_order), so that a wave's utterances share a variant
    CK(hipMalloc(&dhops, sizeof(PlanHop) * (size_t)B * hstride));
    CK(hipMalloc(&dwork, (size_t)plan_work_bytes(B, hstride)));
    PlanArgs pa{dt, df, F, B, hop, 0, T, dplan, 0, 0, &dt->consts.sec[0], dhops, hstride, dwork, true, (int64_t)B * hstride};
    CK(launch_plan_hops(pa, nullptr));
    std::vector<PlanHop> hh((size_t)B * hstride);
    CK(hipMemcpy(hh.data(), dhops, sizeof(PlanHop) * hh.size(), hipMemcpyDeviceToHost));
    std::vector<int32_t> order;
    for (int cls = 0; cls < 3; ++cls)
      for (int u = 0; u < B; ++u) {
        uint64_t m = 0;
        for (int64_t q = 0; q < hstride; ++q) m |= hh[(size_t)u * hstride + q].noise;
        const int c = (m & ~NoiseV<TW, NZ_GLOTTIS>::SERVES) == 0 ? 0 : (m & ~NoiseV<TW, NZ_TONGUE1>::SERVES) == 0 ? 1 : 2;
        if (c == cls) order.push_back(u);
      }
    CK(hipMalloc(&dorder, sizeof(int32_t) * B));
    CK(hipMemcpy(dorder, order.data(), sizeof(int32_t) * B, hipMemcpyHostToDevice));
    a.plan_stride = 0;
    a.hops = dhops;
    a.hop_stride = hstride;
    a.order = dorder;
    a.noise_variants = 1;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, nullptr));
  if (g_hops) hipLaunchKernelGGL(tree_prof_kernel<true>, dim3(blocks), dim3(64 * PWPB), 0, nullptr, a, dprof);
  else hipLaunchKernelGGL(tree_prof_kernel<false>, dim3(blocks), dim3(64 * PWPB), 0, nullptr, a, dprof);
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
  g_wave_ph = h;  // (before the pair kernel's placement slots are cleared)
  // (the pair kernel keeps each wave's placement and span in three slots it does not time)
  for (int w = 0; w < waves; ++w)
    for (int p : {(int)PH_PLACE_HW, (int)PH_PLACE_T0, (int)PH_PLACE_T1}) h[(size_t)w * PH_COUNT + p] = 0;
  for (int w = 0; w < waves; ++w)
    for (int p = 0; p < PH_COUNT; ++p) {
      cycles[p] += h[(size_t)w * PH_COUNT + p];
      g_wave[w] += h[(size_t)w * PH_COUNT + p];
    }
  (void)hipFree(dt); (void)hipFree(df); (void)hipFree(ds); (void)hipFree(dout);
  (void)hipFree(dlds); (void)hipFree(dlanes); (void)hipFree(dprof); (void)hipFree(dplan); (void)hipFree(dp25);
  if (dhops) (void)hipFree(dhops);
  if (dwork) (void)hipFree(dwork);
  if (dorder) (void)hipFree(dorder);
  delete ht;
  return waves;
}
