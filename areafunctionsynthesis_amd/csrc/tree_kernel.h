// tree_kernel.h -- body of the cooperative synthesis kernel (afs_solver AFS_SOLVER_TREE),
// shared by tds_tree.hip (the product kernel) and tools/phase_prof (the same body with
// per-phase cycle counters).
//
// Mapping on gfx950: a wave64 holds four utterances, TREE_W = 16 lanes each.  A lane keeps
// the state of its 6 sections (3 dynamic + 3 static) and their in-currents in registers
// for the whole launch; the four utterances' 8.4 KB LDS blocks carry neighbour exchange,
// the per-sample solver arrays and the small persistent state.  Waves never wait for one
// another (no __syncthreads in the time loop): phases of one utterance are ordered by
// wave-level fences, which is all LDS needs inside a wave.  The time loop runs inside the
// kernel; a launch covers a range of frame transitions and saves the lane/LDS state at the
// end, so long utterances and incremental sessions continue exactly where they stopped.
#pragma once

#include <hip/hip_runtime.h>

#include "afs_tree.h"
#include "tree_core.h"

namespace afs {
namespace tree {

// A DPP lane move whose every lane's source is inside its row (the permutations, rotations and
// broadcasts used here), or whose out-of-row lanes read 0 (bound_ctrl): the destination's old
// value is never kept, so the move carries none (update_dpp(0, ...) zeroed it first: ~90 moves
// per sample, +0.3 % without them, profiles/r03z_ab.txt).
#define AFS_DPP(src, ctrl, rmask, bmask, bc) __builtin_amdgcn_mov_dpp((src), (ctrl), (rmask), (bmask), (bc))

// Lanes per utterance: W = 16 (TREE_W, the throughput kernel: four utterances per wave64, six
// sections per lane) or W = 64 (the voice kernel: one utterance per wave, two sections per lane --
// fewer instructions per sample on the chain, for batches that leave SIMDs idle and for
// real-time voices).  The solver always runs on the utterance's first 16 lanes.
constexpr int TW = TREE_W;
template <int W>
struct Geom {
  static_assert(W == 16 || W == 32 || W == 64, "collectives are written for 16, 32 or 64 lanes per utterance");
  static constexpr int UPW = 64 / W;                 // utterances per wave
  static constexpr int WPB = W == 64 ? 1 : TREE_WPB;  // waves per block (they share one copy of the tables)
  static constexpr int UPB = UPW * WPB;              // utterances per block
};
constexpr int UPW = Geom<TW>::UPW;
constexpr int WPB = Geom<TW>::WPB;
constexpr int UPB = Geom<TW>::UPB;
static_assert(UPB == TREE_UPB, "afs_tree.h TREE_UPB: the host's slot orders group utterances by block");

#ifndef AFS_PAIR_MARK_SB
// the pair kernel: a scheduling barrier at the phase marks whose bit (tree_core.h PH_*) is set (A/B)
#define AFS_PAIR_MARK_SB 0xFFFFFFFFu
#endif
template <bool PROF, int W = TW, bool MARK_SB = false>
struct GpuExec {
  static constexpr bool kToneOut = AFS_TONE_K6 != 0;  // the tone filter in K6 from the stored p[25] (afs_tree.h)
  static constexpr bool kGlottisSplit = true;   // the glottis' masses on the two lane halves (+1.1 %, r03ag_ab.txt)
  int gl;
  Lane<W> *R;
  uint64_t last = 0;
  uint64_t acc[PROF ? PH_COUNT : 1] = {};
  int prio = 0;  // (wave pairs: the launch's STAT priority mode, TreeArgs::stat_prio)
  template <class F> __device__ __forceinline__ void par(F f) { f(gl, *R); }
  // the lane's registers, for values that are the same on every lane of the utterance
  __device__ __forceinline__ const Lane<W> &first() const { return *R; }
  template <class F> __device__ __forceinline__ void one(F f) { if (gl == 0) f(*R); }
  // Per-lane work and lane-uniform work in one block: every lane also evaluates the uniform
  // part (same inputs, same values, same stores), so the two interleave without a branch.
  template <class F, class G> __device__ __forceinline__ void par_uniform(F f, G g) { f(gl, *R); g(*R); }
  template <class F> __device__ __forceinline__ void lanes(int n, F f) {
    if (n >= W || gl < n) f(gl, *R);  // (no branch when every lane takes part)
  }
  __device__ __forceinline__ void sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // the wave pairs' barrier (AFS_PAIR): every wave of the workgroup, LDS visible across them
  // (scheduling barriers around it: the scheduler does not mix the phases' code, which would keep
  // both phases' values live at once -- the pair kernel must fit 256 registers)
  __device__ __forceinline__ void bar() {
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
  }
  // Bit gl of the result: f(gl, R) of this utterance's lane gl.
  template <class F> __device__ __forceinline__ uint64_t ballot(F f) {
    const bool p = f(gl, *R);
    const uint64_t b = __ballot(p);
    if constexpr (W == 64) return b;
    else return (b >> (__lane_id() & ~(W - 1))) & ((1ull << W) - 1);
  }
  template <int CTRL> __device__ __forceinline__ static int dpp(int v) {
    return AFS_DPP(v, CTRL, 0xF, 0xF, false);
  }
  template <int CTRL> __device__ __forceinline__ static double dpp(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const int lo = dpp<CTRL>((int)(uint32_t)b), hi = dpp<CTRL>((int)(uint32_t)(b >> 32));
    return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
  }
  // Areas of the neighbouring dynamic sections: section s = 23 + jW + gl, so s+1 is slot j
  // of lane gl+1 (slot j+1 of lane 0 for the last lane) and s-1 slot j of lane gl-1 (slot
  // j-1 of the last lane for lane 0).  16 lanes: row rotations (row_ror 15 / 1) of the
  // utterance's DPP row; 32 lanes: ds_bpermute.
  __device__ __forceinline__ void dyn_neighbors() {
    using S = Shape<W>;
#pragma unroll
    for (int j = 0; j < S::ND; ++j) {
      const double up = (j + 1 < S::ND) ? R->acur[j + 1 < S::ND ? j + 1 : j] : 0.0;
      const double dn = (j >= 1) ? R->acur[j >= 1 ? j - 1 : j] : 0.0;
      if constexpr (W == 16) {
        const double a = dpp<0x12F>(R->acur[j]), b = dpp<0x12F>(up);  // from lane gl+1 (mod 16)
        const double c = dpp<0x121>(R->acur[j]), d = dpp<0x121>(dn);  // from lane gl-1 (mod 16)
        R->anx[j] = gl == W - 1 ? b : a;
        R->apv[j] = gl == 0 ? d : c;
      } else if constexpr (S::ND == 1) {  // (64 lanes: one dynamic slot, no wrap into another slot)
        const int base = (int)(__lane_id() & ~(W - 1));
        R->anx[j] = __shfl(R->acur[j], base + (gl + 1) % W, 64);
        R->apv[j] = __shfl(R->acur[j], base + (gl + W - 1) % W, 64);
      } else {
        const int base = (int)(__lane_id() & ~(W - 1));
        const int nl = base + (gl + 1) % W, pl = base + (gl + W - 1) % W;
        const double a = __shfl(R->acur[j], nl, 64), b = __shfl(up, nl, 64);
        const double c = __shfl(R->acur[j], pl, 64), d = __shfl(dn, pl, 64);
        R->anx[j] = gl == W - 1 ? b : a;
        R->apv[j] = gl == 0 ? d : c;
      }
    }
  }
  // Inclusive prefix sums over the utterance's lanes: row_shr 1, 2, 4, 8 with zero fill
  // (bound_ctrl) inside the 16-lane row; for 32 lanes, lane 15 of the first row is added to
  // the second (row_bcast15 into rows 1 and 3).  64 lanes: the sums of lanes 16-63 stay row-local
  // -- the only caller (rng_block) consumes lanes < rng_lanes() = 10 alone.
  template <int CTRL> __device__ __forceinline__ static uint32_t shr(uint32_t v) {
    return (uint32_t)AFS_DPP((int)v, CTRL, 0xF, 0xF, true);
  }
  template <int N, class F, class G> __device__ __forceinline__ void scan_add(F f, G g) {
    U4 v = f(gl, *R);
#pragma unroll
    for (int i = 0; i < N; ++i) {
      uint32_t x = v.v[i];
      x += shr<0x111>(x);
      x += shr<0x112>(x);
      x += shr<0x114>(x);
      x += shr<0x118>(x);
      // (rows 1 and 3 only: the other rows keep the old value 0)
      if constexpr (W == 32) x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
      v.v[i] = x;
    }
    g(gl, *R, v);
  }
  // Lane gl+K's value inside the 16-lane row: row_shl K (K > 0) / row_shr -K, zero fill.
  template <int K> __device__ __forceinline__ static double shift(double v) {
    static_assert(K != 0 && K > -16 && K < 16, "row shift");
    constexpr int CTRL = K > 0 ? 0x100 + K : 0x110 - K;
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const int lo = AFS_DPP((int)(uint32_t)b, CTRL, 0xF, 0xF, true);
    const int hi = AFS_DPP((int)(uint32_t)(b >> 32), CTRL, 0xF, 0xF, true);
    return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
  }
  template <int K, int N, class F, class G> __device__ __forceinline__ void pull(F f, G g) {
    const D4 v = f(gl, *R);
    D4 o{{0.0, 0.0, 0.0, 0.0}};
#pragma unroll
    for (int i = 0; i < N; ++i) o.v[i] = shift<K>(v.v[i]);
    g(gl, *R, o);
  }
  // 32-bit forms of pull (lane gl+K's value inside the 16-lane row, zero fill) and of a broadcast
  // of lane K of the row (row_newbcast K), for the rand() stream's double block (rng_block2)
  template <int K, int N, class F, class G> __device__ __forceinline__ void pull_u(F f, G g) {
    static_assert(K != 0 && K > -16 && K < 16, "row shift");
    constexpr int CTRL = K > 0 ? 0x100 + K : 0x110 - K;
    U4 v = f(gl, *R);
#pragma unroll
    for (int i = 0; i < N; ++i) v.v[i] = (uint32_t)AFS_DPP((int)v.v[i], CTRL, 0xF, 0xF, true);
    g(gl, *R, v);
  }
  template <int K, int N, class F, class G> __device__ __forceinline__ void bcast_u(F f, G g) {
    static_assert(K >= 0 && K < 16, "lane of the row");
    U4 v = f(gl, *R);
#pragma unroll
    for (int i = 0; i < N; ++i) v.v[i] = (uint32_t)AFS_DPP((int)v.v[i], 0x150 + K, 0xF, 0xF, false);
    g(gl, *R, v);
  }
  // whether p holds on any lane of the wave (every utterance of it)
  __device__ __forceinline__ static bool wave_any(bool p) { return __ballot(p) != 0; }
  // The lane half (0: lanes 0-7, 1: lanes 8-15 of the utterance) and lane gl ^ 8's value
  // (row_ror 8 inside the 16-lane row), for glottis_eval_split.
  __device__ __forceinline__ int half8() const { return (gl >> 3) & 1; }
  __device__ __forceinline__ static double xch8(double v) { return dpp<0x128>(v); }
  // Word K of this sample's plan (tree_plan.h): lane K of each 16-lane row holds it
  // (R.planw), DPP row_newbcast hands it to the whole row.
  template <int K> __device__ __forceinline__ uint64_t rec() {
    const uint64_t v = R->planw;
    const int lo = AFS_DPP((int)(uint32_t)v, 0x150 + K, 0xF, 0xF, false);
    const int hi = AFS_DPP((int)(uint32_t)(v >> 32), 0x150 + K, 0xF, 0xF, false);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
  }
  // (MARK_SB, the wave pairs: a scheduling barrier at each phase mark -- the scheduler otherwise
  // hoists a phase's loads into the one before and the pair kernel spills)
  __device__ __forceinline__ void mark(int ph) {
    if constexpr (PROF) {
      uint64_t t = __builtin_amdgcn_s_memtime();
      acc[ph] += t - last;
      last = t;
    } else if constexpr (MARK_SB) {
      if ((((uint32_t)AFS_PAIR_MARK_SB) >> ph) & 1u) __builtin_amdgcn_sched_barrier(0);
    }
  }
};

// LDS of one block: the packed hot tables (shared by all its utterances) and one block per
// utterance.
template <int W>
struct WaveLdsT {
  Consts C;
  double X[Geom<W>::UPB][X_STRIDE];
};
using WaveLds = WaveLdsT<TW>;

// The noise-phase variant a wave runs a launch in (tree_core.h NoiseV): the lightest one that
// serves every dipole and constriction any sample of the launch may target -- the or of its
// utterances' hop records (PlanHop::noise, every sample's decisions) -- and every dipole slot that
// still holds amplitude (damp != 0 in the saved lane state: its smoother must keep running).
// Wave-uniform.  Decided before the body loads any state, so that each variant's body (a whole
// copy: tree_synth_body) has live ranges of its own: with the branch between time loops instead,
// the register allocator spilled 160-250 VGPRs of the persistent state to scratch.
template <int W>
__device__ __forceinline__ int noise_variant(const TreeArgs &a, int g = -1, int gl = -1) {
  constexpr int UPB_ = Geom<W>::UPB;
  if (g < 0) {
    g = (int)threadIdx.x / W;
    gl = (int)threadIdx.x % W;
  }
  const int slot = blockIdx.x * UPB_ + g;
  const int u = a.order ? a.order[slot] : slot;
  const int ue = u < a.B ? u : 0;  // (a padding slot runs utterance 0's data and stores nothing)
  const int64_t row = a.frame_row ? a.frame_row[ue] : ue;
  const int64_t nh = (a.s_end - 1) / a.hop - a.s_begin / a.hop + 1;
  const PlanHop *h0 = a.hops + row * a.hop_stride;
  uint64_t m = 0;
  for (int64_t q = gl; q < nh; q += W) m |= h0[q].noise;
  const Lane<W> &L = ((const Lane<W> *)a.lane_state)[(int64_t)ue * W + gl];
#pragma unroll
  for (int k = 0; k < Shape<W>::NDP; ++k)
    if (L.damp[k] != 0.0 && gl + k * W < NDIP) m |= 1ull << (gl + k * W);
#pragma unroll
  for (int o = 32; o >= 1; o /= 2) m |= __shfl_xor(m, o, 64);
  int nz = NZ_FULL;
  if ((AFS_NZ_SET & 4) && (m & ~NoiseV<W, NZ_T1ALL>::SERVES) == 0) nz = NZ_T1ALL;
  if ((AFS_NZ_SET & 1) && (m & ~NoiseV<W, NZ_TONGUE1>::SERVES) == 0) nz = NZ_TONGUE1;
  if ((AFS_NZ_SET & 2) && (m & ~NoiseV<W, NZ_GLOTTIS>::SERVES) == 0) nz = NZ_GLOTTIS;
  const int on = a.variants_dev ? *a.variants_dev : a.noise_variants;
  return __builtin_amdgcn_readfirstlane(on ? nz : (int)NZ_FULL);
}

// AFS_TONE_K6 == 2: the glottal-tone filter (TdsModel.cpp:494-510, 687-705) over positions j0 .. j1
// of a 16-sample output window -- lane p of the utterance's row holds sample p's section-25 pressure
// (wp) and radiated flow (wo) -- in sample order, with K6's operations in K6's order (uncontracted),
// so the audio is the same bit for bit as with the filter in K6; the state (X_TONE) in LDS between
// windows.  Every lane evaluates the recurrence (lane-uniform), lane p keeps its sample's sum.
template <int P, class F> __device__ __forceinline__ void unroll16(F &f) {
  f(std::integral_constant<int, P>{});
  if constexpr (P + 1 < 16) unroll16<P + 1>(f);
}
template <class Ex>
__device__ __forceinline__ void tone_window(int gl, double *X, const Consts &C, int j0, int j1, double &wo,
                                            double wp) {
#pragma clang fp contract(off)
  double x1 = X[X_TONE + 0], x2 = X[X_TONE + 1], x3 = X[X_TONE + 2], x4 = X[X_TONE + 3];
  double y1 = X[X_TONE + 4], y2 = X[X_TONE + 5], y3 = X[X_TONE + 6], y4 = X[X_TONE + 7];
  const double *ta = C.h.tone_a, *tb = C.h.tone_b;
  const double a0 = ta[0], a1 = ta[1], a2 = ta[2], a3 = ta[3], a4 = ta[4];
  const double b1 = tb[1], b2 = tb[2], b3 = tb[3], b4 = tb[4];
  auto step = [&](auto P) {
    constexpr int p = decltype(P)::value;
    if (p < j0 || p > j1) return;
    const double xp = Ex::template dpp<0x150 + p>(wp);  // (row_newbcast p)
    double tacc = a0 * xp;
    tacc += a1 * x1;
    tacc += b1 * y1;
    tacc += a2 * x2;
    tacc += b2 * y2;
    tacc += a3 * x3;
    tacc += b3 * y3;
    tacc += a4 * x4;
    tacc += b4 * y4;
    x4 = x3; x3 = x2; x2 = x1; x1 = xp;
    y4 = y3; y3 = y2; y2 = y1; y1 = tacc;
    wo = gl == p ? wo + tacc : wo;
  };
  unroll16<0>(step);
  if (gl == 0) {
    X[X_TONE + 0] = x1; X[X_TONE + 1] = x2; X[X_TONE + 2] = x3; X[X_TONE + 3] = x4;
    X[X_TONE + 4] = y1; X[X_TONE + 5] = y2; X[X_TONE + 6] = y3; X[X_TONE + 7] = y4;
  }
}

// prof (PROF only): per wave, PH_COUNT cycle sums (s_memtime) over the launch.
// HOPS: the plan words come from hop records (a.hops, tree_plan.h PlanHop): lane gl keeps word
// gl's kind and inputs for the hop and evaluates the word at every sample; a mixed hop's samples
// read their dense records as without HOPS.
template <bool PROF, int MODEL, bool HOPS, int W, int NZ>
__device__ __forceinline__ void tree_synth_run(const TreeArgs &a, WaveLdsT<W> &lds, uint64_t *prof,
                                               int nz = NZ_FULL) {
  constexpr int UPB_ = Geom<W>::UPB, WPB_ = Geom<W>::WPB;
  const int lane = threadIdx.x;  // 0 .. 64 WPB - 1
  const int g = lane / W, gl = lane % W;
  const int slot = blockIdx.x * UPB_ + g;
  const int u = a.order ? a.order[slot] : slot;
  const bool valid = u < a.B;
  const int ue = valid ? u : 0;
  double *X = lds.X[g];
  const Tables &T = *a.tab;
  {  // stage the hot tables (8-byte words; Consts is a multiple of 8 bytes)
    const uint64_t *src = (const uint64_t *)&T.consts;
    uint64_t *dst = (uint64_t *)&lds.C;
    for (int k = lane; k < (int)(sizeof(Consts) / 8); k += 64 * WPB_) dst[k] = src[k];
  }
  Lane<W> R = ((const Lane<W> *)a.lane_state)[(int64_t)ue * W + gl];
  const double *ls = a.lds_state + (int64_t)ue * X_TOTAL;
  for (int k = gl; k < X_TOTAL; k += W) X[k] = ls[k];
  __syncthreads();
  const Consts &C = lds.C;
  GpuExec<PROF, W> ex{gl, &R};
  if constexpr (PROF) ex.last = __builtin_amdgcn_s_memtime();
  const int64_t row = a.frame_row ? a.frame_row[ue] : ue;
  const afs_frame *fu = a.frames + row * a.frame_stride;
  double *o = a.out + (int64_t)ue * a.out_stride;
  double *p25o = a.p25 + (int64_t)ue * a.p25_stride;
  // this utterance's plan records, word gl % 16 of each (tree_plan.h)
  const uint64_t *pl = a.plan + row * a.plan_stride * PLAN_WORDS + (gl & (PLAN_WORDS - 1));
  const int hop = a.hop;
  const int64_t n = a.s_end - a.s_begin;
  int k = (int)(a.s_begin / hop) + 1, i = (int)(a.s_begin % hop);
  // The output stage (dU/dt, Chebyshev low-pass, scaling) and the glottal-tone filter do not feed
  // back into the tube: the kernel stores the radiated flows and section 25's pressures, and K6
  // (tree_output_kernel) filters them after the launch, so none of the filters' state or code is
  // in this kernel's registers.
  frame_load<W>(gl, R, X, fu + (k - 1), fu + k);
  // hop mode: this hop's record (word gl % 16: its kind and inputs; whether the hop is mixed)
  const PlanHop *hr = HOPS ? a.hops + row * a.hop_stride : nullptr;
  double hp[4] = {0.0, 0.0, 0.0, 0.0};
  uint32_t hkind = PK_CONST;
  bool hmixed = !HOPS;
  // a mixed hop's dense records (compact: slot h->dense of a.plan), word gl % 16 of sample 0
  const uint64_t *pd = nullptr;
  auto hop_load = [&](const PlanHop *h) {
    const double2 *q = reinterpret_cast<const double2 *>(h->p[gl & (PLAN_WORDS - 1)]);
    const double2 v0 = q[0], v1 = q[1];
    hp[0] = v0.x; hp[1] = v0.y; hp[2] = v1.x; hp[3] = v1.y;
    hkind = h->kind[gl & (PLAN_WORDS - 1)];
    hmixed = h->mixed != 0;
    pd = a.plan + (int64_t)h->dense * hop * PLAN_WORDS + (gl & (PLAN_WORDS - 1));
  };
  if constexpr (HOPS) hop_load(hr);
  // Dense kernel (hops < 32: target sequences play one frame per sample): the fields of the
  // next right frame are loaded during the last sample of a hop, so that their latency hides
  // behind that sample's work instead of stalling the frame transition; the new left frame is
  // the old right one (frame_shift).
  NextFrame<W> nf{};
  // The per-sample outputs (the radiated flow: every lane has it; section 25's pressure: lane 2's
  // slot 0) are held in a register window of the 16 samples of one 128-byte line of o -- lane j
  // of the utterance keeps the sample at position j of the line; p25o sits at the same position in
  // its lines (afs_capi.cpp lays it out so) -- and lanes 0-15 store the window as one whole line of
  // each array when its last sample is in (or the launch ends): one coalesced store per line
  // instead of 16 single 8-byte stores, which the memory system wrote back as partial lines (2x
  // the stored bytes, profiles/pmc_traffic.json r03aj).  Measured against those stores and against
  // the window in LDS: +0.4 % / +0.5 % (profiles/r04f_store_ab.txt).
  const int o_line = (int)((reinterpret_cast<uintptr_t>(o) >> 3) & 15);
  double wo = 0.0, wp = 0.0;
  const double dhop = (double)hop, inv_hop = 1.0 / dhop;
  ex.sync();
  uint64_t next = hmixed ? (HOPS ? pd[i * PLAN_WORDS] : pl[0]) : 0;
  for (int64_t t = 0; t < n; ++t) {
    // (the ratio at the top of each step -- the next sample's computed at the end of the previous
    // step instead measured -2.5 %, profiles/r03ad_ab.txt; hop_ratio instead of the IEEE division
    // +0.7 %, profiles/r04i_ab.txt)
    const double ratio = hop_ratio(i, dhop, inv_hop);
    const int64_t tn = t + 1 < n ? t + 1 : t;
    if constexpr (HOPS) {
      const uint64_t ev = plan_word_fast(hkind, hp, ratio);
      R.planw = hmixed ? next : ev;
      // (a hop that is not mixed reads its own record's first word: a cache hit, no branch; the
      // load under a branch instead measured the same, profiles/r03w_ab.txt)
      next = *(hmixed ? pd + (i + 1 < hop ? i + 1 : i) * PLAN_WORDS : reinterpret_cast<const uint64_t *>(hr));
    } else {
      R.planw = next;
      next = pl[tn * PLAN_WORDS];  // the next sample's word, a sample ahead
      if (i + 1 == hop && t + 1 < n) nf.load(gl, fu + k + 1);
    }
    sample_step<W, MODEL, NZ>(ex, X, a.uni, C, ratio, true, nz);
    {
      const int j = (o_line + (int)t) & 15;  // the sample's position in its line
      const double p25v = GpuExec<PROF, W>::template dpp<0x152>(R.p[0]);  // lane 2's p[25] to its row
      const bool mine = gl == j;
      wo = mine ? R.sample : wo;
      wp = mine ? p25v : wp;
      if constexpr (AFS_TONE_K6 == 2) {
        // the glottal-tone filter over the window's samples once it is complete (positions j0 .. j),
        // its outputs added to the window's flows before the store (wave-uniform when the utterances'
        // rows are congruent modulo 16 doubles, else per utterance)
        if (j == 15 || t + 1 == n) {
          const int j0 = t >= j ? 0 : (int)(j - t);
          if (a.uni.opt.radiation_from_skin) tone_window<GpuExec<PROF, W>>(gl, X, C, j0, j, wo, wp);
        }
      }
      // lane gl stores window entry gl, sample t - j + gl, if it belongs to this launch
      if (valid && (j == 15 || t + 1 == n) && gl <= j && t - j + gl >= 0) {
        o[t - j + gl] = wo;
        if constexpr (AFS_TONE_K6 == 1) p25o[t - j + gl] = wp;
      }
    }
    if (++i == hop) {
      i = 0;
      ++k;
      if (t + 1 < n) {
        if constexpr (HOPS) {
          // the right frame becomes the left one (registers / LDS), only the new right frame is
          // read: each frame crosses HBM once per utterance instead of twice
          NextFrame<W> f{};
          f.load(gl, fu + k);
          frame_shift<W>(gl, R, X, f);
          hop_load(++hr);
          if (hmixed) next = pd[0];
        } else {
          frame_shift<W>(gl, R, X, nf);
        }
      }
      ex.sync();
    }
  }
  ex.sync();
  if (valid) {
    // (the per-sample fields carry nothing to the next launch; zero them so that their
    // last values are not kept alive through the time loop for this store)
#pragma unroll
    for (int j = 0; j < Shape<W>::ND; ++j) R.acur[j] = R.lcur[j] = R.anx[j] = R.apv[j] = 0.0;
    R.ac = ArmCarry{};
    ((Lane<W> *)a.lane_state)[(int64_t)u * W + gl] = R;
    double *ws = a.lds_state + (int64_t)u * X_TOTAL;
    for (int k = gl; k < X_TOTAL; k += W) ws[k] = X[k];
  }
  if constexpr (PROF) {
    if (lane % 64 == 0)
      for (int p = 0; p < PH_COUNT; ++p)
        prof[((int64_t)blockIdx.x * WPB_ + lane / 64) * PH_COUNT + p] = ex.acc[p];
  }
}

// The kernel body: in hop mode each wave picks its noise-phase variant for the launch
// (noise_variant) and runs the whole body compiled for it.  (The waves of a block may take
// different variants: each reaches the one __syncthreads of the table staging in its own copy.)
#ifndef AFS_NZ_INNER
#define AFS_NZ_INNER 0  // 1: one body, the variant switched in the noise phase (NZ_DYN); 0: a body per variant
#endif
template <bool PROF, int MODEL, bool HOPS = false, int W = TW>
__device__ __forceinline__ void tree_synth_body(const TreeArgs &a, WaveLdsT<W> &lds, uint64_t *prof) {
  // (a launch of the hop-mode fast path whose mixed hops overflowed K5's compact slots: the host runs
  // the call through the chunked path instead, afs_capi.cpp run_chunks)
  if (a.skip_claims && (int64_t)*a.skip_claims > a.skip_cap) return;
  if (a.order) {  // a block of padding slots only (the XCD-dealt slot order) has nothing to do
    bool any = false;
#pragma unroll
    for (int g = 0; g < Geom<W>::UPB; ++g) any |= a.order[blockIdx.x * Geom<W>::UPB + g] < a.B;
    if (!any) return;
  }
  if constexpr (HOPS && AFS_NZ_INNER) {
    tree_synth_run<PROF, MODEL, HOPS, W, NZ_DYN>(a, lds, prof, noise_variant<W>(a));
  } else if constexpr (HOPS) {
    const int nz = noise_variant<W>(a);
    if (false) {
#if AFS_NZ_SET & 2
    } else if (nz == NZ_GLOTTIS) {
      tree_synth_run<PROF, MODEL, HOPS, W, NZ_GLOTTIS>(a, lds, prof);
#endif
#if AFS_NZ_SET & 1
    } else if (nz == NZ_TONGUE1) {
      tree_synth_run<PROF, MODEL, HOPS, W, NZ_TONGUE1>(a, lds, prof);
#endif
#if AFS_NZ_SET & 4
    } else if (nz == NZ_T1ALL) {
      tree_synth_run<PROF, MODEL, HOPS, W, NZ_T1ALL>(a, lds, prof);
#endif
    } else {
      tree_synth_run<PROF, MODEL, HOPS, W, NZ_FULL>(a, lds, prof);
    }
  } else {
    tree_synth_run<PROF, MODEL, HOPS, W, NZ_FULL>(a, lds, prof);
  }
}

// ---------------------------------------------------------------------------
// Wave pairs (AFS_PAIR = 1, an A/B build): a workgroup of four waves for the same eight utterances
// -- waves 0 and 1 take the dynamic slots of utterances 0-3 / 4-7 (ROLE_DYN), waves 2 and 3 their
// static slots and the lane-uniform phases (ROLE_STAT) -- and two workgroups per CU: two waves per
// SIMD, whose instructions the SIMD interleaves (a wave alone issues one VALU instruction per 4
// cycles; the SIMD executes one per 2, tree_core.h sample_step_pair).  Each wave holds half the
// slots' state, so the pair's kernel must fit 256 registers per lane.
// ---------------------------------------------------------------------------
#if AFS_PAIR
// (W = 64: the voice kernel's pairs, one utterance per workgroup of two waves, tree_pair64_body)
template <int MODEL, bool HOPS, int NZ, int ROLE, bool PROF = false, int W = TW>
__device__ __forceinline__ void tree_pair_run(const TreeArgs &a, WaveLdsT<W> &lds, int grp, uint64_t *prof = nullptr) {
  constexpr int UPB_ = Geom<W>::UPB;
  constexpr int NT = 2 * 64 * Geom<W>::WPB;  // threads per workgroup (a pair per wave of the one-wave kernel)
  using S = Shape<W>;
  const int lane = threadIdx.x;  // 0 .. 255
  const int g = grp * Geom<W>::UPW + (lane % 64) / W, gl = lane % W;
  const int slot = blockIdx.x * UPB_ + g;
  const int u = a.order ? a.order[slot] : slot;
  const bool valid = u < a.B;
  const int ue = valid ? u : 0;
  double *X = lds.X[g];
  const Tables &T = *a.tab;
  {
    const uint64_t *src = (const uint64_t *)&T.consts;
    uint64_t *dst = (uint64_t *)&lds.C;
    for (int k = lane; k < (int)(sizeof(Consts) / 8); k += NT) dst[k] = src[k];
  }
  Lane<W> R = ((const Lane<W> *)a.lane_state)[(int64_t)ue * W + gl];
  const double *ls = a.lds_state + (int64_t)ue * X_TOTAL;
  if constexpr (ROLE == ROLE_DYN)
    for (int k = gl; k < X_TOTAL; k += W) X[k] = ls[k];
  __syncthreads();
  const Consts &C = lds.C;
  GpuExec<PROF, W, AFS_PAIR_MARK_SB != 0> ex{gl, &R};
  ex.prio = a.stat_prio;
  const int64_t row = a.frame_row ? a.frame_row[ue] : ue;
  const afs_frame *fu = a.frames + row * a.frame_stride;
  double *o = a.out + (int64_t)ue * a.out_stride;
  double *p25o = a.p25 + (int64_t)ue * a.p25_stride;
  const uint64_t *pl = a.plan + row * a.plan_stride * PLAN_WORDS + (gl & (PLAN_WORDS - 1));
  const int hop = a.hop;
  const int64_t n = a.s_end - a.s_begin;
  int k = (int)(a.s_begin / hop) + 1, i = (int)(a.s_begin % hop);
  if constexpr (ROLE == ROLE_DYN) frame_load<W>(gl, R, X, fu + (k - 1), fu + k);
  const PlanHop *hr = HOPS ? a.hops + row * a.hop_stride : nullptr;
  double hp[4] = {0.0, 0.0, 0.0, 0.0};
  uint32_t hkind = PK_CONST;
  bool hmixed = !HOPS;
  const uint64_t *pd = nullptr;
  auto hop_load = [&](const PlanHop *h) {
    const double2 *q = reinterpret_cast<const double2 *>(h->p[gl & (PLAN_WORDS - 1)]);
    const double2 v0 = q[0], v1 = q[1];
    hp[0] = v0.x; hp[1] = v0.y; hp[2] = v1.x; hp[3] = v1.y;
    hkind = h->kind[gl & (PLAN_WORDS - 1)];
    hmixed = h->mixed != 0;
    pd = a.plan + (int64_t)h->dense * hop * PLAN_WORDS + (gl & (PLAN_WORDS - 1));
  };
  if constexpr (HOPS && ROLE == ROLE_STAT) hop_load(hr);
  NextFrame<W> nf{};
  const int o_line = (int)((reinterpret_cast<uintptr_t>(o) >> 3) & 15);
  double wo = 0.0, wp = 0.0;
  const double dhop = (double)hop, inv_hop = 1.0 / dhop;
#if AFS_PAIR_RNG_DYN
  if constexpr (ROLE == ROLE_STAT) {  // (the ring's head and pending count from the saved lane state)
    if (gl == 0) {
      int32_t *hp = (int32_t *)(X + X_RNGHP);
      hp[0] = R.rhead;
      hp[1] = R.rpend;
    }
  }
#endif
  __syncthreads();  // (the LDS image and X_FRAME in place for both roles)
  uint64_t next = 0;
  if constexpr (ROLE == ROLE_STAT) next = hmixed ? (HOPS ? pd[i * PLAN_WORDS] : pl[0]) : 0;
  if constexpr (ROLE == ROLE_STAT) {
    if (pair_prio(ex) == 3) AFS_SETPRIO(2);  // (the whole launch; modes 1, 2: sample_step_pair)
  }
  uint64_t t_begin = 0;
  if constexpr (PROF) t_begin = ex.last = __builtin_amdgcn_s_memtime();
  for (int64_t t = 0; t < n; ++t) {
    const double ratio = hop_ratio(i, dhop, inv_hop);
    const int64_t tn = t + 1 < n ? t + 1 : t;
    if constexpr (ROLE == ROLE_STAT) {
      if constexpr (HOPS) {
        const uint64_t ev = plan_word_fast(hkind, hp, ratio);
        R.planw = hmixed ? next : ev;
        next = *(hmixed ? pd + (i + 1 < hop ? i + 1 : i) * PLAN_WORDS : reinterpret_cast<const uint64_t *>(hr));
      } else {
        R.planw = next;
        next = pl[tn * PLAN_WORDS];
      }
    } else if constexpr (!HOPS) {
      if (i + 1 == hop && t + 1 < n) nf.load(gl, fu + k + 1);
    }
    sample_step_pair<W, MODEL, NZ, ROLE>(ex, X, a.uni, C, ratio, (int)(t & 1));
    if constexpr (ROLE == ROLE_DYN) {
      const int j = (o_line + (int)t) & 15;
      const double p25v = GpuExec<false, W>::template dpp<0x152>(R.p[0]);
      const bool mine = gl == j;
      wo = mine ? R.sample : wo;
      wp = mine ? p25v : wp;
      if (valid && (j == 15 || t + 1 == n) && gl <= j && t - j + gl >= 0) {
        o[t - j + gl] = wo;
        if constexpr (AFS_TONE_K6 == 1) p25o[t - j + gl] = wp;
      }
    }
    if (++i == hop) {
      i = 0;
      ++k;
      if (t + 1 < n) {
        if constexpr (ROLE == ROLE_DYN) {
          if constexpr (HOPS) {
            NextFrame<W> f{};
            f.load(gl, fu + k);
            frame_shift<W>(gl, R, X, f);
          } else {
            frame_shift<W>(gl, R, X, nf);
          }
        } else if constexpr (HOPS) {
          hop_load(++hr);
          if (hmixed) next = pd[0];
        }
      }
      ex.bar();
    }
    ex.mark(PH_TAIL);
  }
  if constexpr (PROF) {
    // (the wave's placement -- HW_ID, XCC_ID -- and its loop's span, for tools/phase_prof)
    ex.acc[PH_PLACE_HW] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                          ((uint64_t)(__builtin_amdgcn_s_getreg((15 << 11) | 20) & 15) << 32);
    ex.acc[PH_PLACE_T0] = t_begin;
    ex.acc[PH_PLACE_T1] = __builtin_amdgcn_s_memtime();
    if (lane % 64 == 0)
      for (int q = 0; q < PH_COUNT; ++q) prof[((int64_t)blockIdx.x * (NT / 64) + lane / 64) * PH_COUNT + q] = ex.acc[q];
  }
  if constexpr (ROLE == ROLE_DYN) {  // (the displacements of the last sample into X_RELX, the image's slot)
    if (n & 1) {
      if (gl < 4) X[X_RELX + gl] = X[X_RELX2 + gl];
    }
  }
  __syncthreads();
  if (valid) {
    Lane<W> *dst = (Lane<W> *)a.lane_state + (int64_t)u * W + gl;
#pragma unroll
    for (int j = 0; j < S::NSL; ++j) {
      if (!role_slot<ROLE>(j, S::ND)) continue;
      dst->p[j] = R.p[j]; dst->pr[j] = R.pr[j]; dst->w[j] = R.w[j]; dst->wr[j] = R.wr[j];
      dst->wr2[j] = R.wr2[j]; dst->u[j] = R.u[j]; dst->ur[j] = R.ur[j]; dst->un[j] = R.un[j];
    }
    if constexpr (ROLE == ROLE_DYN) {
#pragma unroll
      for (int j = 0; j < S::ND; ++j) {
        dst->aL[j] = R.aL[j]; dst->aR[j] = R.aR[j]; dst->lL[j] = R.lL[j]; dst->lR[j] = R.lR[j];
        dst->al[j] = R.al[j]; dst->be[j] = R.be[j];
      }
      double *ws = a.lds_state + (int64_t)u * X_TOTAL;
      for (int q = gl; q < X_TOTAL; q += W) ws[q] = X[q];
    } else {
#pragma unroll
      for (int q = 0; q < S::NDP; ++q) {
        dst->damp[q] = R.damp[q]; dst->dout[q] = R.dout[q]; dst->dcut[q] = R.dcut[q]; dst->racc[q] = R.racc[q];
      }
#if AFS_PAIR_RNG_DYN
      const int32_t *hp = (const int32_t *)(X + X_RNGHP);
      dst->rhead = hp[0];
      dst->rpend = hp[1];
#else
      dst->rhead = R.rhead;
      dst->rpend = R.rpend;
#endif
    }
  }
}

// The two workgroups a compute unit holds at a time (AFS_PAIR_MAP 3): each claims one of two slots
// in its CU's word (global atomics; released when the workgroup ends).
__device__ unsigned int pair_cu_slots[2048];

// Roles: two groups of four utterances; in each group one wave is DYN and one STAT.  The SIMD a wave
// runs on decides (AFS_PAIR_MAP 3), so that each SIMD runs one DYN and one STAT wave of its CU's two
// workgroups -- STAT carries the targets, noise and solver, the longer half: two STAT waves on one
// SIMD would share its issue slots.  When a workgroup's four waves do not sit on four SIMDs, or
// under the other maps, by the wave index (0: waves 0, 1 DYN; 1: a slot parity read from
// HW_ID.WAVE_ID; 2: the block's parity).  Any placement gives a valid pairing; this only balances
// the SIMDs.
template <int MODEL, bool HOPS, bool PROF = false>
__device__ __forceinline__ void tree_pair_body(const TreeArgs &a, WaveLdsT<TW> &lds, int *pattern,
                                               uint64_t *prof = nullptr) {
  if (a.skip_claims && (int64_t)*a.skip_claims > a.skip_cap) return;
  if (a.order) {
    bool any = false;
#pragma unroll
    for (int g = 0; g < Geom<TW>::UPB; ++g) any |= a.order[blockIdx.x * Geom<TW>::UPB + g] < a.B;
    if (!any) return;
  }
  const int wave = (int)threadIdx.x / 64;
#ifndef AFS_PAIR_MAP
// 3: by SIMD and the CU's workgroup slot; 0: waves 0, 1 DYN (groups 0, 1), 2, 3 STAT; 1: by the wave
// slot's parity; 2: by the block's parity (profiles/r06_pair_ab.txt)
#define AFS_PAIR_MAP 3
#endif
  int grp, st;
  unsigned int *cu_word = nullptr;
  unsigned int cu_bit = 0;
  if constexpr (AFS_PAIR_MAP == 0) {
    grp = wave & 1;
    st = wave >> 1;
  } else if constexpr (AFS_PAIR_MAP == 3) {
    const unsigned int hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_ID
    const int simd = (int)((hw >> 4) & 3);
    if (threadIdx.x % 64 == 0) pattern[1 + wave] = simd;
    if (threadIdx.x == 0) {
      const unsigned int xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20) & 7;  // XCC_ID
      cu_word = pair_cu_slots + ((xcc << 8) | ((hw >> 8) & 255));              // SE, SH, CU
      const unsigned int old = atomicOr(cu_word, 1u);
      cu_bit = 1u;
      if (old & 1u) {
        const unsigned int o2 = atomicOr(cu_word, 2u);
        cu_bit = (o2 & 2u) ? 0u : 2u;
      }
      pattern[0] = cu_bit == 2u;
    }
    __syncthreads();
    const int m = (1 << pattern[1]) | (1 << pattern[2]) | (1 << pattern[3]) | (1 << pattern[4]);
    if (m == 15) {
      grp = simd & 1;
      st = (simd >> 1) ^ pattern[0];
    } else {
      grp = wave & 1;
      st = (wave >> 1) ^ pattern[0];
    }
  } else {
    if (threadIdx.x == 0)
      *pattern = AFS_PAIR_MAP == 1 ? (int)(__builtin_amdgcn_s_getreg((3 << 11) | 4) & 1)  // HW_ID.WAVE_ID bit 0
                                   : (int)(blockIdx.x & 1);
    __syncthreads();
    grp = wave >> 1;
    st = (wave & 1) ^ *pattern;
  }
  const bool stat = st != 0;
#ifdef AFS_PAIR_PROBE  // (register probes: 1 compiles the DYN role alone, 2 the STAT role's NZ_FULL copy alone)
  if constexpr (AFS_PAIR_PROBE == 1) { tree_pair_run<MODEL, HOPS, NZ_FULL, ROLE_DYN, PROF>(a, lds, grp, prof); return; }
  if constexpr (AFS_PAIR_PROBE == 2) { tree_pair_run<MODEL, HOPS, NZ_FULL, ROLE_STAT, PROF>(a, lds, grp, prof); return; }
#endif
  if (!stat) {
    tree_pair_run<MODEL, HOPS, NZ_FULL, ROLE_DYN, PROF>(a, lds, grp, prof);
  } else if constexpr (HOPS) {
    const int g = grp * Geom<TW>::UPW + ((int)threadIdx.x % 64) / TW, gl = (int)threadIdx.x % TW;
    const int nz = noise_variant<TW>(a, g, gl);
    if (false) {
#if AFS_NZ_SET & 2
    } else if (nz == NZ_GLOTTIS) {
      tree_pair_run<MODEL, HOPS, NZ_GLOTTIS, ROLE_STAT, PROF>(a, lds, grp, prof);
#endif
#if AFS_NZ_SET & 1
    } else if (nz == NZ_TONGUE1) {
      tree_pair_run<MODEL, HOPS, NZ_TONGUE1, ROLE_STAT, PROF>(a, lds, grp, prof);
#endif
    } else {
      tree_pair_run<MODEL, HOPS, NZ_FULL, ROLE_STAT, PROF>(a, lds, grp, prof);
    }
  } else {
    tree_pair_run<MODEL, HOPS, NZ_FULL, ROLE_STAT, PROF>(a, lds, grp, prof);
  }
  if constexpr (AFS_PAIR_MAP == 3) {
    if (threadIdx.x == 0 && cu_bit) atomicAnd(cu_word, ~cu_bit);  // (after the run's last workgroup barrier)
  }
}

// The voice kernel's pairs (64 lanes per utterance): one utterance per workgroup of two waves, wave 0
// DYN and wave 1 STAT, for batches that leave a SIMD to each wave (afs_tree.h TREE_PAIR64_MAX): the
// sample's chain split over two SIMDs instead of one wave's.
template <int MODEL, bool HOPS, bool PROF = false>
__device__ __forceinline__ void tree_pair64_body(const TreeArgs &a, WaveLdsT<64> &lds, uint64_t *prof = nullptr) {
  if (a.skip_claims && (int64_t)*a.skip_claims > a.skip_cap) return;
  if (a.order && a.order[blockIdx.x] >= a.B) return;
  const bool stat = threadIdx.x >= 64;
  if (!stat) {
    tree_pair_run<MODEL, HOPS, NZ_FULL, ROLE_DYN, PROF, 64>(a, lds, 0, prof);
  } else if constexpr (HOPS) {
    const int nz = noise_variant<64>(a, 0, (int)threadIdx.x % 64);
    if (false) {
#if AFS_NZ_SET & 2
    } else if (nz == NZ_GLOTTIS) {
      tree_pair_run<MODEL, HOPS, NZ_GLOTTIS, ROLE_STAT, PROF, 64>(a, lds, 0, prof);
#endif
#if AFS_NZ_SET & 1
    } else if (nz == NZ_TONGUE1) {
      tree_pair_run<MODEL, HOPS, NZ_TONGUE1, ROLE_STAT, PROF, 64>(a, lds, 0, prof);
#endif
    } else {
      tree_pair_run<MODEL, HOPS, NZ_FULL, ROLE_STAT, PROF, 64>(a, lds, 0, prof);
    }
  } else {
    tree_pair_run<MODEL, HOPS, NZ_FULL, ROLE_STAT, PROF, 64>(a, lds, 0, prof);
  }
}

#endif  // AFS_PAIR

}  // namespace tree
}  // namespace afs
