// seg_kernel.h -- body of the segment-aligned synthesis kernel (afs_solver AFS_SOLVER_SEG),
// shared by tds_seg.hip and development tools.
//
// Mapping on gfx950: a wave64 holds four utterances, sixteen lanes (one DPP row) each.  Lane gl
// of an utterance owns the dynamic and static slots of seg_model.h's partition in every phase
// of the sample; the state of its sections and currents stays in registers for the whole
// launch, its LDS block carries only the values another lane's row or the noise sources read
// (the source sections' terms, the solution, the noise-smoothed flows) and the small state.
// Cross-lane steps are DPP row operations; phases of one utterance are ordered by wave-level
// fences (no __syncthreads in the time loop).  A launch covers a range of samples and saves the
// lane / LDS state at its end.
#pragma once

#include <hip/hip_runtime.h>

#include "afs_seg.h"
#include "seg_core.h"

namespace afs {
namespace seg {

constexpr int UPW = 64 / SW;          // utterances per wave
constexpr int WPB = AFS_SEG_WPB;      // waves per block (they share one copy of the tables)
constexpr int UPB = UPW * WPB;        // utterances per block

template <bool PROF>
struct SegGpuExec {
  int gl;
  SegLane *R;
  uint64_t last = 0;
  uint64_t acc[PROF ? 8 : 1] = {};
  template <class F> __device__ __forceinline__ void par(F f) { f(gl, *R); }
  template <class F, class G> __device__ __forceinline__ void par_uniform(F f, G g) { f(gl, *R); g(*R); }
  __device__ __forceinline__ void sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  __device__ __forceinline__ void mark(int ph) {
    if constexpr (PROF) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      acc[ph & 7] += t - last;
      last = t;
    }
  }
  template <int CTRL, bool BC> __device__ __forceinline__ static double dpp(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, 0xF, 0xF, BC);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), CTRL, 0xF, 0xF, BC);
    return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
  }
  template <int CTRL> __device__ __forceinline__ static uint64_t dpp64(uint64_t v) {
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, 0xF, 0xF, false);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
  }
  // word K of this sample's plan: lane K of each row holds it, row_newbcast hands it to the row
  template <int K> __device__ __forceinline__ uint64_t rec() { return dpp64<0x150 + K>(R->planw); }
  template <class F> __device__ __forceinline__ uint64_t ballot(F f) {
    const bool p = f(gl, *R);
    const uint64_t b = __ballot(p);
    return (b >> (__lane_id() & ~(SW - 1))) & ((1ull << SW) - 1);
  }
  // OR over the row: quad_perm xor 1, xor 2, row_half_mirror, row_mirror
  template <class F> __device__ __forceinline__ uint64_t or64(F f) {
    uint64_t v = f(gl, *R);
    v |= dpp64<0xB1>(v);
    v |= dpp64<0x4E>(v);
    v |= dpp64<0x141>(v);
    v |= dpp64<0x140>(v);
    return v;
  }
  template <int CTRL> __device__ __forceinline__ static uint32_t shr(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, true);
  }
  template <int N, class F, class G> __device__ __forceinline__ void scan_add(F f, G g) {
    tree::U4 v = f(gl, *R);
#pragma unroll
    for (int i = 0; i < N; ++i) {
      uint32_t x = v.v[i];
      x += shr<0x111>(x);
      x += shr<0x112>(x);
      x += shr<0x114>(x);
      x += shr<0x118>(x);
      v.v[i] = x;
    }
    g(gl, *R, v);
  }
  // lane gl+K's values inside the row (zero outside): row_shl K / row_shr -K, bound_ctrl
  template <int K, int N, class F, class G> __device__ __forceinline__ void pull(F f, G g) {
    static_assert(K != 0 && K > -16 && K < 16, "row shift");
    constexpr int CTRL = K > 0 ? 0x100 + K : 0x110 - K;
    const tree::D4 v = f(gl, *R);
    tree::D4 o{{0.0, 0.0, 0.0, 0.0}};
#pragma unroll
    for (int i = 0; i < N; ++i) o.v[i] = dpp<CTRL, true>(v.v[i]);
    g(gl, *R, o);
  }
  // lane K's values to the whole row (row_newbcast)
  template <int K, int N, class F, class G> __device__ __forceinline__ void bcast(F f, G g) {
    const tree::D4 v = f(gl, *R);
    tree::D4 o{{0.0, 0.0, 0.0, 0.0}};
#pragma unroll
    for (int i = 0; i < N; ++i) o.v[i] = dpp<0x150 + K, false>(v.v[i]);
    g(gl, *R, o);
  }
};

struct SegWaveLds {
  SegHot H;
  SegConsts C;
  double X[UPB][SX_STRIDE];
};

template <bool PROF, int MODEL>
__device__ __forceinline__ void seg_synth_body(const SegArgs &sa, SegWaveLds &lds, uint64_t *prof) {
  const TreeArgs &a = sa.t;
  const int lane = threadIdx.x;
  const int g = lane / SW, gl = lane % SW;
  const int u = blockIdx.x * UPB + g;
  const bool valid = u < a.B;
  const int ue = valid ? u : 0;
  double *X = lds.X[g];
  const Tables &T = *a.tab;
  {  // stage the lane records and the scalars (8-byte words)
    const uint64_t *src = (const uint64_t *)&sa.seg->c;
    uint64_t *dst = (uint64_t *)&lds.C;
    for (int k = lane; k < (int)(sizeof(SegConsts) / 8); k += 64 * WPB) dst[k] = src[k];
    const uint64_t *hs = (const uint64_t *)&T.consts.h;
    uint64_t *hd = (uint64_t *)&lds.H.h;
    static_assert(sizeof(Hot) % 8 == 0, "Hot: 8-byte words");
    for (int k = lane; k < (int)(sizeof(Hot) / 8); k += 64 * WPB) hd[k] = hs[k];
  }
  SegLane R = ((const SegLane *)a.lane_state)[(int64_t)ue * SW + gl];
  const double *ls = a.lds_state + (int64_t)ue * SX_TOTAL;
  for (int k = gl; k < SX_TOTAL; k += SW) X[k] = ls[k];
  if (gl < GB && gl != G_D) X[SX_G + GB * (S_LAST_TRACHEA - G0) + gl] = sa.seg->g22[gl];
  __syncthreads();
  const SegConsts &C = lds.C;
  SegGpuExec<PROF> ex{gl, &R};
  if constexpr (PROF) ex.last = __builtin_amdgcn_s_memtime();
  const int64_t row = a.frame_row ? a.frame_row[ue] : ue;
  const afs_frame *fu = a.frames + row * a.frame_stride;
  double *o = a.out + (int64_t)ue * a.out_stride;
  const uint64_t *pl = a.plan + row * a.plan_stride * tree::PLAN_WORDS + (gl & (tree::PLAN_WORDS - 1));
  const int hop = a.hop;
  const int64_t n = a.s_end - a.s_begin;
  int k = (int)(a.s_begin / hop) + 1, i = (int)(a.s_begin % hop);
  const bool defer = hop >= tree::OUT_DEFER_MIN_HOP;
  seg_frame_load(gl, R, X, C, fu + (k - 1), fu + k);
  ex.sync();
  uint64_t next = pl[0];
  int64_t t0 = 0;
  for (int64_t t = 0; t < n; ++t) {
    R.planw = next;
    next = pl[(t + 1 < n ? t + 1 : t) * tree::PLAN_WORDS];  // the next sample's word, a sample ahead
    const double ratio = (double)i / (double)hop;
#if defined(AFS_SEG_OPAQUE)
    // (the tables' addresses opaque per sample: their loads stay in the loop instead of holding
    // registers for the whole launch)
    const SegConsts *cp = &C;
    __asm__ volatile("" : "+s"(cp));
    seg_sample_step<MODEL>(ex, X, a.uni, lds.H, *cp, ratio, defer);
#else
    seg_sample_step<MODEL>(ex, X, a.uni, lds.H, C, ratio, defer);
#endif
    if (valid && gl == 0) o[t] = R.sample;
    if (++i == hop) {
      if (defer && valid && gl == 0) seg_output_filter_run(X, lds.H, o + t0, (int)(t + 1 - t0));
      t0 = t + 1;
      i = 0;
      ++k;
      if (t + 1 < n) seg_frame_load(gl, R, X, C, fu + (k - 1), fu + k);
      ex.sync();
    }
  }
  if (defer && valid && gl == 0 && t0 < n) seg_output_filter_run(X, lds.H, o + t0, (int)(n - t0));
  ex.sync();
  if (valid) {
    R.k = SegWork{};  // (per-sample values carry nothing to the next launch)
    ((SegLane *)a.lane_state)[(int64_t)u * SW + gl] = R;
    double *ws = a.lds_state + (int64_t)u * SX_TOTAL;
    for (int q = gl; q < SX_TOTAL; q += SW) ws[q] = X[q];
  }
  if constexpr (PROF) {
    if (lane % 64 == 0)
      for (int p = 0; p < 8; ++p) prof[((int64_t)blockIdx.x * WPB + lane / 64) * 8 + p] = ex.acc[p];
  }
}

}  // namespace seg
}  // namespace afs
