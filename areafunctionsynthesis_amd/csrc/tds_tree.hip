// tds_tree.hip -- the cooperative synthesis kernel (afs_solver AFS_SOLVER_TREE); the body and
// the wave mapping are described in tree_kernel.h.
#include "tree_kernel.h"

namespace afs {

using namespace tree;

namespace {

__global__ void __launch_bounds__(64 * WPB, AFS_TREE_MIN_WAVES) tree_synth_kernel(TreeArgs a) {
  __shared__ WaveLds lds;
  tree_synth_body<false>(a, lds, nullptr);
}

__global__ void tree_reset_kernel(Lane<TW> *lanes, double *lds, int B, const uint32_t *seeds) {
  const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (int64_t)B * TW) return;
  const int u = (int)(id / TW), gl = (int)(id % TW);
  Lane<TW> R;
  reset_lane<TW>(gl, R);
  lanes[id] = R;
  if (gl == 0) reset_lds(lds + (int64_t)u * X_TOTAL, seeds ? seeds[u] : 1u);
}

__global__ void tree_nonfinite_kernel(const double *lds, int B, int32_t *count) {
  int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= B) return;
  if (lds[(int64_t)u * X_TOTAL + X_NONFIN] != 0.0) atomicAdd(count, 1);
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
  if (a.B <= 0 || a.k_end <= a.k_begin) return hipSuccess;
  hipLaunchKernelGGL(tree_synth_kernel, dim3((a.B + UPB - 1) / UPB), dim3(64 * WPB), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_tree_nonfinite(const double *lds_state, int B, int32_t *count, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(tree_nonfinite_kernel, dim3((B + 63) / 64), dim3(64), 0, st, lds_state, B, count);
  return hipGetLastError();
}

}  // namespace afs
