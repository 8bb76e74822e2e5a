// tds_tree.hip -- the cooperative synthesis kernel (afs_solver AFS_SOLVER_TREE) and the
// small state kernels; the body and the wave mapping are described in tree_kernel.h.  (Its
// noise-source plan kernel K5 is in tds_plan.hip.)
#include "tree_kernel.h"

namespace afs {

using namespace tree;

namespace {

// one kernel per glottis model (TriangularGlottis, the reference's; TwoMassModel), plan mode
// (HOPS: hop records, hops >= PLAN_HOP_MIN; dense records otherwise) and lanes per utterance W
// (16: the throughput kernel; 64: the voice kernel, tree_kernel.h)
template <int MODEL, bool HOPS, int W>
__global__ void __launch_bounds__(64 * Geom<W>::WPB, AFS_TREE_MIN_WAVES) tree_synth_kernel(TreeArgs a) {
  __shared__ WaveLdsT<W> lds;
  tree_synth_body<false, MODEL, HOPS, W>(a, lds, nullptr);
}

#if AFS_PAIR
// the wave-pair build of the throughput kernel (tree_kernel.h tree_pair_body): four waves per
// workgroup, two per SIMD
template <int MODEL, bool HOPS>
__global__ void __launch_bounds__(256, 2) tree_pair_kernel(TreeArgs a) {
  __shared__ WaveLdsT<TW> lds;
  __shared__ int pattern[5];
  tree_pair_body<MODEL, HOPS>(a, lds, pattern);
}
// the voice kernel's pairs: two waves per utterance, each may take a whole SIMD's registers
template <int MODEL, bool HOPS>
__global__ void __launch_bounds__(128, AFS_PAIR64_WAVES) tree_pair64_kernel(TreeArgs a) {
  __shared__ WaveLdsT<64> lds;
  tree_pair64_body<MODEL, HOPS>(a, lds);
}
#endif

// K6: the output stage of a launch's samples -- dU/dt, the 8-pole Chebyshev low-pass, x 0.004 /
// 32767 (Synthesizer.cpp:614-627) -- over the radiated flows the synthesis kernel stored, in
// place, one thread per utterance; the filter state (X_OUTF, X_PREVFLOW, X_NONFIN, X_TONE) lives in
// the utterance's saved LDS image, which the synthesis kernel carries through unchanged.  With skin
// radiation (TdsModel::Options.radiationFromSkin): first the glottal-tone filter over section 25's
// stored pressures, added to the flows, in the output filter's loop (tone_output_run).
__global__ void __launch_bounds__(64) tree_output_kernel(const Tables *tab, double *lds_state, double *out,
                                                         int64_t out_stride, int64_t n, int B, const double *p25,
                                                         int64_t p25_stride, int skin,
                                                         const uint32_t *skip_claims, int64_t skip_cap) {
  const int u = blockIdx.x * 64 + threadIdx.x;
  if (u >= B) return;
  if (skip_claims && (int64_t)*skip_claims > skip_cap) return;  // (as the guarded K1 launch: TreeArgs)
  double *X = lds_state + (int64_t)u * X_TOTAL;
  double *o = out + (int64_t)u * out_stride;
  if (p25 && skin) tone_output_run(X, tab->consts, p25 + (int64_t)u * p25_stride, o, (int)n);
  else output_filter_run(X, tab->consts, o, (int)n);
}

// seeds == nullptr: utterance u is seeded u + 1 (afs.h)
template <int W>
__global__ void tree_reset_kernel(Lane<W> *lanes, double *lds, int B, const uint32_t *seeds) {
  const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (int64_t)B * W) return;
  const int u = (int)(id / W), gl = (int)(id % W);
  Lane<W> R;
  reset_lane<W>(gl, R);
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

// Diagnostics (afs_tube_interpolate): the synthesis kernel's own frame_load + phase_interpolate,
// compiled in this file with its flags, for n (frame pair, ratio) samples; thread (i, gl) writes
// the pharynx/mouth sections of lane gl's slots.  X: a private stand-in of the LDS block's frame
// values (only X_FRAME .. X_FRAME + 3 are read).
__global__ void tree_interp_kernel(const Tables *tab, const afs_frame *fl, const afs_frame *fr, const double *ratio,
                                   int n, double *area, double *len) {
  const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (int64_t)n * TW) return;
  const int i = (int)(id / TW), gl = (int)(id % TW);
  Lane<TW> R = Lane<TW>{};
  double X[X_FRAME + 16];
  for (int k = 0; k < X_FRAME + 16; ++k) X[k] = 0.0;
  frame_load<TW>(0, R, X, fl + i, fr + i);  // (lane 0's frame values for every thread)
  frame_load<TW>(gl, R, X, fl + i, fr + i);
  phase_interpolate<TW>(gl, R, X, tab->consts, ratio[i]);
#pragma unroll
  for (int j = 0; j < Shape<TW>::ND; ++j) {
    const int m = dyn_section(TW, j, gl) - S_PHARYNX0;
    if (m >= 0 && m < NPM) {
      area[(int64_t)i * NPM + m] = R.acur[j];
      len[(int64_t)i * NPM + m] = R.lcur[j];
    }
  }
}

// Diagnostics (afs_plan_hop_words): the synthesis kernel's per-sample plan words, plan_word_fast
// compiled here with its flags, for n (hop record, ratio) pairs: thread (i, w) writes word w.
__global__ void tree_hop_words_kernel(const tree::PlanHop *h, const double *ratio, int n, uint64_t *out) {
  const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (int64_t)n * PLAN_WORDS) return;
  const int i = (int)(id / PLAN_WORDS), w = (int)(id % PLAN_WORDS);
  out[id] = plan_word_fast(h[i].kind[w], h[i].p[w], ratio[i]);
}

}  // namespace

hipError_t launch_tree_hop_words(const tree::PlanHop *h, const double *ratio, int n, uint64_t *out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t t = (int64_t)n * PLAN_WORDS;
  hipLaunchKernelGGL(tree_hop_words_kernel, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, st, h, ratio, n, out);
  return hipGetLastError();
}

hipError_t launch_tree_interp(const Tables *tab, const afs_frame *fl, const afs_frame *fr, const double *ratio, int n,
                              double *area, double *len, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t t = (int64_t)n * TW;
  hipLaunchKernelGGL(tree_interp_kernel, dim3((unsigned)((t + 127) / 128)), dim3(128), 0, st, tab, fl, fr, ratio, n,
                     area, len);
  return hipGetLastError();
}

hipError_t launch_tree_output(const Tables *tab, double *lds_state, double *out, int64_t out_stride, int64_t n, int B,
                              const double *p25, int64_t p25_stride, int skin, hipStream_t st,
                              const uint32_t *skip_claims, int64_t skip_cap) {
  if (B <= 0 || n <= 0) return hipSuccess;
  hipLaunchKernelGGL(tree_output_kernel, dim3((B + 63) / 64), dim3(64), 0, st, tab, lds_state, out, out_stride, n, B,
                     p25, p25_stride, skin, skip_claims, skip_cap);
  return hipGetLastError();
}

int64_t tree_lane_bytes(int lanes) { return lanes == 64 ? (int64_t)sizeof(Lane<64>) : (int64_t)sizeof(Lane<TW>); }
int64_t tree_lds_doubles() { return X_TOTAL; }

hipError_t launch_tree_reset(void *lane_state, double *lds_state, int B, const uint32_t *seeds, int lanes,
                             hipStream_t st) {
  if (B <= 0) return hipSuccess;
  const int64_t n = (int64_t)B * lanes;
  const dim3 grid((unsigned)((n + 255) / 256)), block(256);
  if (lanes == 64)
    hipLaunchKernelGGL(tree_reset_kernel<64>, grid, block, 0, st, (Lane<64> *)lane_state, lds_state, B, seeds);
  else
    hipLaunchKernelGGL(tree_reset_kernel<TW>, grid, block, 0, st, (Lane<TW> *)lane_state, lds_state, B, seeds);
  return hipGetLastError();
}

// the one-wave kernel (every phase on one wave)
template <int W>
static void launch_one_wave(const TreeArgs &a, dim3 grid, dim3 block, bool two, hipStream_t st) {
  if (a.hops) {
    if (two) hipLaunchKernelGGL((tree_synth_kernel<AFS_GLOTTIS_TWO_MASS, true, W>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((tree_synth_kernel<AFS_GLOTTIS_TRIANGULAR, true, W>), grid, block, 0, st, a);
  } else {
    if (two) hipLaunchKernelGGL((tree_synth_kernel<AFS_GLOTTIS_TWO_MASS, false, W>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((tree_synth_kernel<AFS_GLOTTIS_TRIANGULAR, false, W>), grid, block, 0, st, a);
  }
}

template <int W>
static void launch_synth_w(const TreeArgs &a, hipStream_t st) {
  constexpr int UPB_ = Geom<W>::UPB;
  const dim3 grid(a.grid_blocks > 0 ? a.grid_blocks : (a.B + UPB_ - 1) / UPB_), block(64 * Geom<W>::WPB);
  const bool two = a.uni.opt.glottis_model == AFS_GLOTTIS_TWO_MASS;
#if AFS_PAIR
  if constexpr (W == TW) {  // (the one-wave kernel at 16 lanes is not instantiated in this build)
    static_assert(Geom<TW>::WPB == 2, "a wave pair per four utterances: 4 waves per 8-utterance block");
    const dim3 pblock(256);
    if (a.hops) {
      if (two) hipLaunchKernelGGL((tree_pair_kernel<AFS_GLOTTIS_TWO_MASS, true>), grid, pblock, 0, st, a);
      else hipLaunchKernelGGL((tree_pair_kernel<AFS_GLOTTIS_TRIANGULAR, true>), grid, pblock, 0, st, a);
    } else {
      if (two) hipLaunchKernelGGL((tree_pair_kernel<AFS_GLOTTIS_TWO_MASS, false>), grid, pblock, 0, st, a);
      else hipLaunchKernelGGL((tree_pair_kernel<AFS_GLOTTIS_TRIANGULAR, false>), grid, pblock, 0, st, a);
    }
  } else if constexpr (W == 64) {
    if (a.B <= TREE_PAIR64_MAX) {
      const dim3 pblock(128);
      if (a.hops) {
        if (two) hipLaunchKernelGGL((tree_pair64_kernel<AFS_GLOTTIS_TWO_MASS, true>), grid, pblock, 0, st, a);
        else hipLaunchKernelGGL((tree_pair64_kernel<AFS_GLOTTIS_TRIANGULAR, true>), grid, pblock, 0, st, a);
      } else {
        if (two) hipLaunchKernelGGL((tree_pair64_kernel<AFS_GLOTTIS_TWO_MASS, false>), grid, pblock, 0, st, a);
        else hipLaunchKernelGGL((tree_pair64_kernel<AFS_GLOTTIS_TRIANGULAR, false>), grid, pblock, 0, st, a);
      }
      return;
    }
  }
  if constexpr (W != TW) launch_one_wave<W>(a, grid, block, two, st);
#else
  launch_one_wave<W>(a, grid, block, two, st);
#endif
}

hipError_t launch_tree_synth(const TreeArgs &a, int lanes, hipStream_t st) {
  if (a.B <= 0 || a.s_end <= a.s_begin) return hipSuccess;
  if (lanes == 64) launch_synth_w<64>(a, st);
  else launch_synth_w<TW>(a, st);
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

// Loads this file's code object on the context's device now (HIP loads a code object at the first
// launch of one of its kernels otherwise: tens of milliseconds inside a real-time caller's first
// buffer).
template <class K> static hipError_t preload_one(K k) {
  hipFuncAttributes at;
  return hipFuncGetAttributes(&at, reinterpret_cast<const void *>(k));
}
hipError_t preload_tree_kernels() {
  hipError_t e = hipSuccess;
  for (hipError_t x : {
#if AFS_PAIR
                       preload_one(tree_pair_kernel<AFS_GLOTTIS_TRIANGULAR, true>),
                       preload_one(tree_pair_kernel<AFS_GLOTTIS_TRIANGULAR, false>),
                       preload_one(tree_pair_kernel<AFS_GLOTTIS_TWO_MASS, true>),
                       preload_one(tree_pair_kernel<AFS_GLOTTIS_TWO_MASS, false>),
                       preload_one(tree_pair64_kernel<AFS_GLOTTIS_TRIANGULAR, true>),
                       preload_one(tree_pair64_kernel<AFS_GLOTTIS_TRIANGULAR, false>),
                       preload_one(tree_pair64_kernel<AFS_GLOTTIS_TWO_MASS, true>),
                       preload_one(tree_pair64_kernel<AFS_GLOTTIS_TWO_MASS, false>),
#else
                       preload_one(tree_synth_kernel<AFS_GLOTTIS_TRIANGULAR, true, TW>),
                       preload_one(tree_synth_kernel<AFS_GLOTTIS_TRIANGULAR, false, TW>),
                       preload_one(tree_synth_kernel<AFS_GLOTTIS_TWO_MASS, true, TW>),
                       preload_one(tree_synth_kernel<AFS_GLOTTIS_TWO_MASS, false, TW>),
#endif
                       preload_one(tree_synth_kernel<AFS_GLOTTIS_TRIANGULAR, true, 64>),
                       preload_one(tree_synth_kernel<AFS_GLOTTIS_TRIANGULAR, false, 64>),
                       preload_one(tree_synth_kernel<AFS_GLOTTIS_TWO_MASS, true, 64>),
                       preload_one(tree_synth_kernel<AFS_GLOTTIS_TWO_MASS, false, 64>),
                       preload_one(tree_output_kernel), preload_one(tree_reset_kernel<TW>),
                       preload_one(tree_reset_kernel<64>), preload_one(tree_nonfinite_kernel),
                       preload_one(tree_draws_kernel)})
    if (e == hipSuccess) e = x;
  return e;
}

}  // namespace afs
