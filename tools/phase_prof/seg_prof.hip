// seg_prof.hip -- development tool: the seg kernel body (seg_kernel.h) with per-phase cycle
// counters (s_memtime deltas of seg_core.h's x.mark, accumulated per wave).  Not part of
// libafs; built by this directory's Makefile and driven by seg_run.py on the GPU box.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "seg_kernel.h"

using namespace afs;
using namespace afs::seg;

__global__ void __launch_bounds__(64 * WPB, 1) seg_prof_kernel(SegArgs a, uint64_t *prof) {
  __shared__ SegWaveLds lds;
  seg_synth_body<true, AFS_GLOTTIS_TRIANGULAR>(a, lds, prof);
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return -1;                                                               \
    }                                                                          \
  } while (0)

constexpr int NPH = 8;
extern "C" int sp_phase_count() { return NPH; }

// frames[B][F] host; cycles[NPH] = sum over waves; returns the wave count, kernel ms in *ms.
extern "C" int sp_run(const afs_frame *frames, const uint32_t *seeds, int B, int F, int hop, double fs,
                      uint64_t *cycles, double *ms) {
  Tables *ht = new Tables();
  build_tables(ht, fs, afs::default_options());
  SegTables *hs = new SegTables();
  build_seg_tables(*ht, hs);
  if (!hs->ok) return -2;
  Tables *dt;
  SegTables *dsg;
  afs_frame *df;
  uint32_t *ds;
  double *dout, *dlds;
  void *dlanes;
  uint64_t *dprof;
  const int blocks = (B + UPB - 1) / UPB, waves = blocks * WPB;
  CK(hipMalloc(&dt, sizeof(Tables)));
  CK(hipMemcpy(dt, ht, sizeof(Tables), hipMemcpyHostToDevice));
  CK(hipMalloc(&dsg, sizeof(SegTables)));
  CK(hipMemcpy(dsg, hs, sizeof(SegTables), hipMemcpyHostToDevice));
  CK(hipMalloc(&df, sizeof(afs_frame) * B * F));
  CK(hipMemcpy(df, frames, sizeof(afs_frame) * B * F, hipMemcpyHostToDevice));
  CK(hipMalloc(&ds, 4 * B));
  CK(hipMemcpy(ds, seeds, 4 * B, hipMemcpyHostToDevice));
  CK(hipMalloc(&dout, sizeof(double) * (size_t)B * (F - 1) * hop));
  CK(hipMalloc(&dlds, sizeof(double) * (size_t)B * seg_lds_doubles()));
  CK(hipMalloc(&dlanes, (size_t)B * SW * seg_lane_bytes()));
  CK(hipMalloc(&dprof, sizeof(uint64_t) * waves * NPH));
  CK(hipMemset(dprof, 0, sizeof(uint64_t) * waves * NPH));
  CK(launch_seg_reset(dlanes, dlds, B, ds, nullptr));
  const int64_t T = (int64_t)(F - 1) * hop;
  uint64_t *dplan;
  CK(hipMalloc(&dplan, (size_t)B * T * PLAN_RECORD_BYTES));
  PlanArgs pa{dt, df, F, B, hop, 0, T, dplan, T, 0, &dsg->uo[0]};
  CK(launch_plan(pa, nullptr));
  SegArgs a{TreeArgs{dt, df, F, nullptr, hop, 0, T, dout, T, dplan, T, dlanes, dlds, B, ht->uni}, dsg};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, nullptr));
  hipLaunchKernelGGL(seg_prof_kernel, dim3(blocks), dim3(64 * WPB), 0, nullptr, a, dprof);
  CK(hipGetLastError());
  CK(hipEventRecord(e1, nullptr));
  CK(hipEventSynchronize(e1));
  float fms = 0;
  CK(hipEventElapsedTime(&fms, e0, e1));
  *ms = fms;
  std::vector<uint64_t> h((size_t)waves * NPH);
  CK(hipMemcpy(h.data(), dprof, sizeof(uint64_t) * h.size(), hipMemcpyDeviceToHost));
  for (int p = 0; p < NPH; ++p) cycles[p] = 0;
  for (int w = 0; w < waves; ++w)
    for (int p = 0; p < NPH; ++p) cycles[p] += h[(size_t)w * NPH + p];
  (void)hipFree(dt); (void)hipFree(dsg); (void)hipFree(df); (void)hipFree(ds); (void)hipFree(dout);
  (void)hipFree(dlds); (void)hipFree(dlanes); (void)hipFree(dprof); (void)hipFree(dplan);
  delete ht;
  delete hs;
  return waves;
}
