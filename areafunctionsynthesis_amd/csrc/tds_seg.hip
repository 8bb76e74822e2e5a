// tds_seg.hip -- the segment-aligned synthesis kernel (afs_solver AFS_SOLVER_SEG) and its small
// state kernels; the body and the wave mapping are described in seg_kernel.h, the partition in
// seg_model.h.  (Its noise-source plans come from K5, tds_plan.hip, with the seg layout's
// offsets.)
#include "seg_kernel.h"

namespace afs {

using namespace seg;

namespace {

template <int MODEL>
__global__ void __launch_bounds__(64 * WPB, 1) seg_synth_kernel(SegArgs a) {
  __shared__ SegWaveLds lds;
  seg_synth_body<false, MODEL>(a, lds, nullptr);
}

// seeds == nullptr: utterance u is seeded u + 1 (afs.h)
__global__ void seg_reset_kernel(SegLane *lanes, double *lds, int B, const uint32_t *seeds) {
  const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (int64_t)B * SW) return;
  const int u = (int)(id / SW), gl = (int)(id % SW);
  SegLane R;
  seg_reset_lane(R);
  lanes[id] = R;
  if (gl == 0) seg_reset_lds(lds + (int64_t)u * SX_TOTAL, seeds ? seeds[u] : (uint32_t)u + 1u);
}

__global__ void seg_nonfinite_kernel(const double *lds, int B, int32_t *count, uint8_t *flags) {
  int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= B) return;
  const bool nf = lds[(int64_t)u * SX_TOTAL + SX_NONFIN] != 0.0;
  if (flags) flags[u] = nf ? 1 : 0;
  if (nf) atomicAdd(count, 1);
}

__global__ void seg_draws_kernel(const double *lds, int B, int64_t *draws) {
  int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= B) return;
  draws[u] = (int64_t)*(const uint64_t *)(lds + (int64_t)u * SX_TOTAL + SX_NDRAW);
}

}  // namespace

int64_t seg_lane_bytes() { return (int64_t)sizeof(SegLane); }
int64_t seg_lds_doubles() { return SX_TOTAL; }

hipError_t launch_seg_reset(void *lane_state, double *lds_state, int B, const uint32_t *seeds, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  int64_t n = (int64_t)B * SW;
  hipLaunchKernelGGL(seg_reset_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, (SegLane *)lane_state,
                     lds_state, B, seeds);
  return hipGetLastError();
}

hipError_t launch_seg_synth(const SegArgs &a, hipStream_t st) {
  if (a.t.B <= 0 || a.t.s_end <= a.t.s_begin) return hipSuccess;
  if (a.t.uni.opt.glottis_model == AFS_GLOTTIS_TWO_MASS)
    hipLaunchKernelGGL(seg_synth_kernel<AFS_GLOTTIS_TWO_MASS>, dim3((a.t.B + UPB - 1) / UPB), dim3(64 * WPB), 0, st, a);
  else
    hipLaunchKernelGGL(seg_synth_kernel<AFS_GLOTTIS_TRIANGULAR>, dim3((a.t.B + UPB - 1) / UPB), dim3(64 * WPB), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_seg_nonfinite(const double *lds_state, int B, int32_t *count, uint8_t *flags, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(seg_nonfinite_kernel, dim3((B + 63) / 64), dim3(64), 0, st, lds_state, B, count, flags);
  return hipGetLastError();
}

hipError_t launch_seg_draws(const double *lds_state, int B, int64_t *draws, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(seg_draws_kernel, dim3((B + 63) / 64), dim3(64), 0, st, lds_state, B, draws);
  return hipGetLastError();
}

}  // namespace afs
