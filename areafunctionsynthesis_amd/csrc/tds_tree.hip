// tds_tree.hip -- the cooperative synthesis kernel (afs_solver AFS_SOLVER_TREE).
//
// Mapping on gfx950: a wave64 holds four utterances, TREE_W = 16 lanes each.  A lane keeps
// the state of its 6 sections (3 dynamic + 3 static) and their in-currents in registers
// for the whole launch; the four utterances' 8.4 KB LDS blocks carry neighbour exchange,
// the per-sample solver arrays and the small persistent state.  Waves never wait for one
// another (no __syncthreads): phases of one utterance are ordered by wave-level fences,
// which is all LDS needs inside a wave.  The time loop runs inside the kernel; a launch
// covers a range of frame transitions and saves the lane/LDS state at the end, so long
// utterances and incremental sessions continue exactly where they stopped.
#include <hip/hip_runtime.h>

#include "afs_tree.h"
#include "tree_core.h"

namespace afs {

using namespace tree;

namespace {

constexpr int TW = TREE_W;
constexpr int UPW = 64 / TW;  // utterances per wave

struct GpuExec {
  int gl;
  Lane<TW> *R;
  template <class F> __device__ __forceinline__ void par(F f) { f(gl, *R); }
  template <class F> __device__ __forceinline__ void one(F f) { if (gl == 0) f(*R); }
  template <class F> __device__ __forceinline__ void lanes(int n, F f) { if (gl < n) f(gl, *R); }
  __device__ __forceinline__ void sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
};

// One block of LDS per wave: the packed hot tables (shared by the four utterances) and the
// four utterance blocks.
struct WaveLds {
  Consts C;
  double X[UPW][X_TOTAL];
};

__global__ void __launch_bounds__(64) tree_synth_kernel(TreeArgs a) {
  __shared__ WaveLds lds;
  const int lane = threadIdx.x;
  const int g = lane / TW, gl = lane % TW;
  const int u = blockIdx.x * UPW + g;
  const bool valid = u < a.B;
  const int ue = valid ? u : 0;
  double *X = lds.X[g];
  const Tables &T = *a.tab;
  {  // stage the hot tables (8-byte words; Consts is a multiple of 8 bytes)
    const uint64_t *src = (const uint64_t *)&T.consts;
    uint64_t *dst = (uint64_t *)&lds.C;
    for (int k = lane; k < (int)(sizeof(Consts) / 8); k += 64) dst[k] = src[k];
  }
  Lane<TW> R = ((const Lane<TW> *)a.lane_state)[(int64_t)ue * TW + gl];
  const double *ls = a.lds_state + (int64_t)ue * X_TOTAL;
  for (int k = gl; k < X_TOTAL; k += TW) X[k] = ls[k];
  __syncthreads();
  const Consts &C = lds.C;
  GpuExec ex{gl, &R};
  const afs_frame *fu = a.frames + (int64_t)ue * a.frame_stride;
  double *o = a.out + (int64_t)ue * a.out_stride;
  int64_t t = 0;
  for (int k = a.k_begin; k < a.k_end; ++k) {
    frame_load<TW>(gl, R, X, fu + (k - 1), fu + k);
    ex.sync();
    for (int i = 0; i < a.hop; ++i) {
      const double ratio = (double)i / (double)a.hop;
      sample_step<TW>(ex, X, T, C, ratio);
      if (valid && gl == 0) o[t] = R.sample;
      ++t;
    }
  }
  ex.sync();
  if (valid) {
    ((Lane<TW> *)a.lane_state)[(int64_t)u * TW + gl] = R;
    double *ws = a.lds_state + (int64_t)u * X_TOTAL;
    for (int k = gl; k < X_TOTAL; k += TW) ws[k] = X[k];
  }
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
  hipLaunchKernelGGL(tree_synth_kernel, dim3((a.B + UPW - 1) / UPW), dim3(64), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_tree_nonfinite(const double *lds_state, int B, int32_t *count, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(tree_nonfinite_kernel, dim3((B + 63) / 64), dim3(64), 0, st, lds_state, B, count);
  return hipGetLastError();
}

}  // namespace afs
