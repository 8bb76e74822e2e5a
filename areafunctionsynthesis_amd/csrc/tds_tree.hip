// tds_tree.hip -- the cooperative synthesis kernel (afs_solver AFS_SOLVER_TREE) and the
// small state kernels; the body and the wave mapping are described in tree_kernel.h.  (Its
// noise-source plan kernel K5 is in tds_plan.hip.)
#include "tree_kernel.h"

namespace afs {

using namespace tree;

namespace {

// one kernel per glottis model (TriangularGlottis, the reference's; TwoMassModel)
template <int MODEL>
__global__ void __launch_bounds__(64 * WPB, AFS_TREE_MIN_WAVES) tree_synth_kernel(TreeArgs a) {
  __shared__ WaveLds lds;
  tree_synth_body<false, MODEL>(a, lds, nullptr);
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
  if (a.uni.opt.glottis_model == AFS_GLOTTIS_TWO_MASS)
    hipLaunchKernelGGL(tree_synth_kernel<AFS_GLOTTIS_TWO_MASS>, dim3((a.B + UPB - 1) / UPB), dim3(64 * WPB), 0, st, a);
  else
    hipLaunchKernelGGL(tree_synth_kernel<AFS_GLOTTIS_TRIANGULAR>, dim3((a.B + UPB - 1) / UPB), dim3(64 * WPB), 0, st, a);
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
