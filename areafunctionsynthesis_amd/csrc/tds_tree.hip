// tds_tree.hip -- the cooperative synthesis kernel (afs_solver AFS_SOLVER_TREE), its
// noise-source plan kernel (K5, tree_plan.h) and the small state kernels; the body and the
// wave mapping are described in tree_kernel.h.
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

// Grid (rows, sample blocks of PLAN_BLOCK): one thread per (frame row, sample), a block of
// consecutive samples of one row.  When the block's samples span at most PLAN_STAGE frames
// (hops >= 128), the frames are staged in LDS first: the plan's scans read every section's
// area / length / articulator several times, and from LDS those reads cost a fraction of the
// cache-hit latency of global loads.  Shorter hops (target sequences, hop 1) read the frames
// from global memory.  The block's records are contiguous in memory: they are assembled in LDS
// and written with one 16-byte store per lane and step over the whole range (a thread's own
// 128-B record written directly would spread each store instruction over 64 lines).
constexpr int PLAN_BLOCK = 256, PLAN_STAGE = 4, PLAN_PITCH = PLAN_WORDS + 1;  // (odd pitch: fewer bank conflicts)
constexpr int FRAME_WORDS = (int)(sizeof(afs_frame) / 8);
static_assert(sizeof(afs_frame) % 8 == 0, "frames are copied as 8-byte words");

__global__ void __launch_bounds__(PLAN_BLOCK) plan_kernel(PlanArgs a) {
  __shared__ uint64_t fr_lds[PLAN_STAGE][FRAME_WORDS];
  __shared__ uint64_t rec_lds[PLAN_BLOCK * PLAN_PITCH];
  const int64_t n = a.s_end - a.s_begin;
  const int64_t row = blockIdx.x;
  const int64_t t_first = (int64_t)blockIdx.y * PLAN_BLOCK;
  const int64_t t_last = (t_first + PLAN_BLOCK < n ? t_first + PLAN_BLOCK : n) - 1;
  const int64_t t = t_first + threadIdx.x;
  const afs_frame *f = a.frames + row * a.frame_stride;
  // sample s plays frames s / hop and s / hop + 1
  const int64_t k_lo = (a.s_begin + t_first) / a.hop, k_hi = (a.s_begin + t_last) / a.hop + 1;
  const bool staged = k_hi - k_lo + 1 <= PLAN_STAGE;  // uniform over the block
  if (staged) {
    const uint64_t *src = (const uint64_t *)(f + k_lo);
    const int words = (int)(k_hi - k_lo + 1) * FRAME_WORDS;
    for (int w = threadIdx.x; w < words; w += PLAN_BLOCK) (&fr_lds[0][0])[w] = src[w];
    __syncthreads();
  }
  if (t < n) {
    const int64_t s = a.s_begin + t;
    const int64_t k = s / a.hop + 1;
    const int i = (int)(s - (k - 1) * a.hop);
    const afs_frame *fl = staged ? (const afs_frame *)fr_lds[k - 1 - k_lo] : f + (k - 1);
    const afs_frame *fr = staged ? (const afs_frame *)fr_lds[k - k_lo] : f + k;
    uint64_t w[PLAN_WORDS];
    plan_sample(fl, fr, (double)i / (double)a.hop, a.tab->consts.sec, a.two_mass != 0, w);
#pragma unroll
    for (int q = 0; q < PLAN_WORDS; ++q) rec_lds[threadIdx.x * PLAN_PITCH + q] = w[q];
  }
  __syncthreads();
  // the block's (t_last - t_first + 1) records, 16 bytes per lane and step
  const int chunks = (int)(t_last - t_first + 1) * (PLAN_WORDS / 2);
  ulonglong2 *o = (ulonglong2 *)(a.plan + (row * a.plan_stride + t_first) * PLAN_WORDS);
  for (int c = threadIdx.x; c < chunks; c += PLAN_BLOCK) {
    const int r = c / (PLAN_WORDS / 2), q = 2 * (c % (PLAN_WORDS / 2));
    o[c] = make_ulonglong2(rec_lds[r * PLAN_PITCH + q], rec_lds[r * PLAN_PITCH + q + 1]);
  }
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

hipError_t launch_plan(const PlanArgs &a, hipStream_t st) {
  const int64_t n = a.s_end - a.s_begin;
  if (n <= 0 || a.rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(plan_kernel, dim3((unsigned)a.rows, (unsigned)((n + PLAN_BLOCK - 1) / PLAN_BLOCK)),
                     dim3(PLAN_BLOCK), 0, st, a);
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
