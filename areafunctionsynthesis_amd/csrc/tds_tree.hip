// tds_tree.hip -- the cooperative synthesis kernel (afs_solver AFS_SOLVER_TREE), its
// noise-source plan kernel (K5, tree_plan.h) and the small state kernels; the body and the
// wave mapping are described in tree_kernel.h.
#include "tree_kernel.h"

namespace afs {

using namespace tree;

namespace {

__global__ void __launch_bounds__(64 * WPB, AFS_TREE_MIN_WAVES) tree_synth_kernel(TreeArgs a) {
  __shared__ WaveLds lds;
  tree_synth_body<false>(a, lds, nullptr);
}

// One thread per (frame row, sample); consecutive threads take consecutive samples of a row,
// so a wave reads the same two frames (cache hits) and writes 64 contiguous records.
__global__ void __launch_bounds__(256) plan_kernel(PlanArgs a) {
  const int64_t n = a.s_end - a.s_begin;
  const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (int64_t)a.rows * n) return;
  const int64_t row = id / n, t = id - row * n, s = a.s_begin + t;
  const int k = (int)(s / a.hop) + 1, i = (int)(s % a.hop);
  const afs_frame *f = a.frames + row * a.frame_stride;
  uint64_t w[PLAN_WORDS];
  plan_sample(f + (k - 1), f + k, (double)i / (double)a.hop, a.tab->consts.sec, a.two_mass != 0, w);
  ulonglong2 *o = (ulonglong2 *)(a.plan + (row * a.plan_stride + t) * PLAN_WORDS);
#pragma unroll
  for (int q = 0; q < PLAN_WORDS / 2; ++q) o[q] = make_ulonglong2(w[2 * q], w[2 * q + 1]);
}

// seeds == nullptr: utterance u is seeded u + 1 (afs.h)
__global__ void tree_reset_kernel(Lane<TW> *lanes, double *lds, int B, const uint32_t *seeds) {
  const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (int64_t)B * TW) return;
  const int u = (int)(id / TW), gl = (int)(id % TW);
  Lane<TW> R;
  reset_lane<TW>(gl, R);
  lanes[id] = R;
  if (gl == 0) reset_lds(lds + (int64_t)u * X_TOTAL, seeds ? seeds[u] : (uint32_t)u + 1u);
}

__global__ void tree_nonfinite_kernel(const double *lds, int B, int32_t *count, uint8_t *flags) {
  int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= B) return;
  const bool nf = lds[(int64_t)u * X_TOTAL + X_NONFIN] != 0.0;
  if (flags) flags[u] = nf ? 1 : 0;
  if (nf) atomicAdd(count, 1);
}

__global__ void tree_draws_kernel(const double *lds, int B, int64_t *draws) {
  int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= B) return;
  draws[u] = (int64_t)*(const uint64_t *)(lds + (int64_t)u * X_TOTAL + X_NDRAW);
}

}  // namespace

int64_t tree_lane_bytes() { return (int64_t)sizeof(Lane<TW>); }
int64_t tree_lds_doubles() { return X_TOTAL; }

hipError_t launch_tree_reset(void *lane_state, double *lds_state, int B, const uint32_t *seeds, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  int64_t n = (int64_t)B * TW;
  hipLaunchKernelGGL(tree_reset_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     (Lane<TW> *)lane_state, lds_state, B, seeds);
  return hipGetLastError();
}

hipError_t launch_tree_synth(const TreeArgs &a, hipStream_t st) {
  if (a.B <= 0 || a.s_end <= a.s_begin) return hipSuccess;
  hipLaunchKernelGGL(tree_synth_kernel, dim3((a.B + UPB - 1) / UPB), dim3(64 * WPB), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_plan(const PlanArgs &a, hipStream_t st) {
  const int64_t n = (int64_t)a.rows * (a.s_end - a.s_begin);
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(plan_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_tree_nonfinite(const double *lds_state, int B, int32_t *count, uint8_t *flags, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(tree_nonfinite_kernel, dim3((B + 63) / 64), dim3(64), 0, st, lds_state, B, count, flags);
  return hipGetLastError();
}

hipError_t launch_tree_draws(const double *lds_state, int B, int64_t *draws, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(tree_draws_kernel, dim3((B + 63) / 64), dim3(64), 0, st, lds_state, B, draws);
  return hipGetLastError();
}

}  // namespace afs
