// tds_plan.hip -- the noise-source plan kernel (K5): the constriction scans of every sample
// ahead of the time loop (tree_plan.h), one thread per (frame row, sample).  A file of its own
// so that it is compiled with its own flags (build.py).
#include "afs_tree.h"
#include "tree_plan.h"

namespace afs {

using namespace tree;

namespace {

// Grid (rows, sample blocks of PLAN_BLOCK): one thread per (frame row, sample), a block of
// consecutive samples of one row.  When the block's samples span at most PLAN_STAGE frames
// (hops >= 128), the frames are staged in LDS first: the plan's scans read every section's
// area / length / articulator several times, and from LDS those reads cost a fraction of the
// cache-hit latency of global loads.  Shorter hops (target sequences, hop 1) read the frames
// from global memory.  Each thread stores its own 128-B record with eight 16-byte stores (the
// block's records are contiguous; L2 merges the partial lines): no LDS for the records, so a K5
// block (4.3 KB of LDS, 80 VGPRs) fits on a CU beside the synthesis kernel's block, which K5 of
// the next launch runs concurrently with (afs_capi.cpp run_chunks).  Assembling the records in
// LDS first for one coalesced store per lane and step measured within 2 %.
#ifndef AFS_PLAN_BLOCK
#define AFS_PLAN_BLOCK 256
#endif
constexpr int PLAN_BLOCK = AFS_PLAN_BLOCK, PLAN_STAGE = 4;
constexpr int FRAME_WORDS = (int)(sizeof(afs_frame) / 8);
static_assert(sizeof(afs_frame) % 8 == 0, "frames are copied as 8-byte words");

__global__ void __launch_bounds__(PLAN_BLOCK) plan_kernel(PlanArgs a) {
  __shared__ uint64_t fr_lds[PLAN_STAGE][FRAME_WORDS];
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
    // the areas clamped once per frame (Tube::setPharynxMouthGeometry's MIN_AREA, idempotent)
    // instead of twice per sample and section
    for (int q = threadIdx.x; q < (int)(k_hi - k_lo + 1) * NPM; q += PLAN_BLOCK) {
      double *ar = ((afs_frame *)fr_lds[q / NPM])->area_cm2 + q % NPM;
      *ar = plan_clampA(*ar);
    }
    __syncthreads();
  }
  if (t < n) {
    const int64_t s = a.s_begin + t;
    const int64_t k = s / a.hop + 1;
    const int i = (int)(s - (k - 1) * a.hop);
    const double ratio = (double)i / (double)a.hop;
    uint64_t w[PLAN_WORDS];
    // two instantiations of the scans: LDS frames (ds_read) and global frames (global loads);
    // one pointer that may point at either would make every frame read a flat load
    if (staged)
      plan_sample<true>((const afs_frame *)fr_lds[k - 1 - k_lo], (const afs_frame *)fr_lds[k - k_lo], ratio, a.uo,
                        a.two_mass != 0, w);
    else
      plan_sample(f + (k - 1), f + k, ratio, a.uo, a.two_mass != 0, w);
    ulonglong2 *o = (ulonglong2 *)(a.plan + (row * a.plan_stride + t) * PLAN_WORDS);
#pragma unroll
    for (int q = 0; q < PLAN_WORDS / 2; ++q) o[q] = make_ulonglong2(w[2 * q], w[2 * q + 1]);
  }
}

// Hop mode (hops >= PLAN_HOP_MIN), two kernels.
// plan_hop_iv_kernel: one thread per (frame row, hop slot) decides the hop's samples inside the
// launch with one evaluation on the interval geometry (tree_plan.h plan_hop_decide_iv).  When
// every comparison is decided for all of them -- static and slowly moving tubes, almost every
// hop -- it writes the hop record (plan_hop_inputs); otherwise (a decision changes within the
// hop or comes too close to call, or the aspiration strength changes) it appends the hop to
// the work list.
// plan_hop_wave_kernel: one wave per work-list hop, persistent over the list.  The hop's two
// frames are staged in LDS (areas clamped once); lane L decides the samples L, L + 64, ... (the
// scans of plan_kernel without the doubles) and compares each decision with the first sample's.
// Lane 0 builds the hop record in LDS, the wave stores it; a mixed hop's samples also get their
// dense records.  Both match the host reference plan_hop_host (per-sample decisions) bit for bit
// (tests/test_plan_gpu.py).
constexpr int HOP_WAVE = 64, HOP_IV_BLOCK = 64;
constexpr int HOP_WORDS = (int)(sizeof(PlanHop) / 8);

struct HopRange {
  int64_t h;       // hop index: frames h, h + 1
  int i0, i1;      // the hop's samples inside the launch
};
__device__ __forceinline__ HopRange hop_range(const PlanArgs &a, int64_t slot) {
  const int64_t h = a.s_begin / a.hop + slot;
  const int64_t s_lo = h * a.hop > a.s_begin ? h * a.hop : a.s_begin;
  const int64_t s_hi = (h + 1) * a.hop < a.s_end ? (h + 1) * a.hop : a.s_end;
  return HopRange{h, (int)(s_lo - h * a.hop), (int)(s_hi - h * a.hop)};
}

// The block's frames -- consecutive (row, hop) ids read a contiguous run of frames when the rows'
// hops are their whole trajectories (frame_stride = slots + 1: every frame-driven call) -- are
// staged in LDS with coalesced loads and their areas clamped once: each thread's decisions read
// its two frames' sections several times over (four scans), and from global memory, one 1072-B
// record per lane, those reads missed the caches -- 9.9 GB of fetch per step of 8192 x 1 s for
// 0.89 GB of frames (profiles/pmc_traffic.json r04ad).  Blocks whose frames are not one short
// run (chunked launches) read them from global memory as before.
constexpr int HOP_IV_STAGE = HOP_IV_BLOCK + 2;  // frames: one more than the block's hops, + a row step

__global__ void __launch_bounds__(HOP_IV_BLOCK) plan_hop_iv_kernel(PlanArgs a, int64_t slots) {
  __shared__ uint64_t fr_lds[HOP_IV_STAGE][FRAME_WORDS];
  const int64_t n_ids = (int64_t)a.rows * slots;
  const int64_t id0 = (int64_t)blockIdx.x * HOP_IV_BLOCK, id = id0 + threadIdx.x;
  const int64_t idl = (id0 + HOP_IV_BLOCK < n_ids ? id0 + HOP_IV_BLOCK : n_ids) - 1;
  // the frame index (into a.frames) of an id's left frame
  auto left = [&](int64_t q) { return (q / slots) * a.frame_stride + a.s_begin / a.hop + q % slots; };
  const int64_t f0 = left(id0), f1 = left(idl) + 1;  // the run the block's frames lie in
  const bool staged = f1 - f0 + 1 <= HOP_IV_STAGE;  // (uniform over the block)
  if (staged) {
    const uint64_t *src = (const uint64_t *)(a.frames + f0);
    const int words = (int)(f1 - f0 + 1) * FRAME_WORDS;
    for (int w = threadIdx.x; w < words; w += HOP_IV_BLOCK) (&fr_lds[0][0])[w] = src[w];
    __syncthreads();
    for (int q = threadIdx.x; q < (int)(f1 - f0 + 1) * NPM; q += HOP_IV_BLOCK) {
      double *ar = ((afs_frame *)fr_lds[q / NPM])->area_cm2 + q % NPM;
      *ar = plan_clampA(*ar);
    }
    __syncthreads();
  }
  if (id >= n_ids) return;
  const int64_t row = id / slots, slot = id % slots;
  const HopRange r = hop_range(a, slot);
  PlanKey k;
  bool ok;
  const afs_frame *fl, *fr;
  if (staged) {  // (two instantiations of the scans: LDS frames, areas clamped, and global frames)
    fl = (const afs_frame *)fr_lds[left(id) - f0];
    fr = fl + 1;
    ok = plan_hop_decide_iv<true>(fl, fr, a.hop, r.i0, r.i1, k);
  } else {
    fl = a.frames + left(id);
    fr = fl + 1;
    ok = plan_hop_decide_iv<false>(fl, fr, a.hop, r.i0, r.i1, k);
  }
  if (ok) {
    PlanHop &h = a.hops[row * a.hop_stride + slot];
    h = PlanHop{};
    ok = plan_hop_inputs(k, fl, fr, a.uo, a.two_mass != 0, h);  // (clampA is idempotent on staged areas)
  }
  if (!ok) a.work[2 + atomicAdd(a.work, 1u)] = (uint32_t)id;
}

__global__ void __launch_bounds__(HOP_WAVE) plan_hop_wave_kernel(PlanArgs a, int64_t slots) {
  __shared__ uint64_t fr_lds[2][FRAME_WORDS];
  __shared__ uint64_t hop_lds[HOP_WORDS];
  const int lane = threadIdx.x;
  const uint32_t nwork = a.work[0];
  for (uint32_t e = blockIdx.x; e < nwork; e += gridDim.x) {
    const uint32_t id = a.work[2 + e];
    const int64_t row = id / slots, slot = id % slots;
    const HopRange r = hop_range(a, slot);
    const int64_t h = r.h;
    const afs_frame *f = a.frames + row * a.frame_stride;
    {
      const uint64_t *src = (const uint64_t *)(f + h);
      for (int w = lane; w < 2 * FRAME_WORDS; w += HOP_WAVE) (&fr_lds[0][0])[w] = src[w];
      __syncthreads();
      for (int q = lane; q < 2 * NPM; q += HOP_WAVE) {
        double *ar = ((afs_frame *)fr_lds[q / NPM])->area_cm2 + q % NPM;
        *ar = plan_clampA(*ar);
      }
      __syncthreads();
    }
    const afs_frame *fl = (const afs_frame *)fr_lds[0], *fr = (const afs_frame *)fr_lds[1];
    const int i0 = r.i0, i1 = r.i1;
    PlanKey k0{};
    uint64_t q0[2] = {0, 0}, noise = 0;
    bool diff = false;
    for (int i = i0 + lane, it = 0; it == 0 || i < i1; i += HOP_WAVE, ++it) {
      uint64_t q[2] = {0, 0};
      PlanKey k{};
      if (i < i1) {
        const double ratio = (double)i / (double)a.hop;
        const PlanGeomT<true> g{fl, fr, 1.0 - ratio, ratio};
        double obst[4], po[4];
        plan_decide(g, k, obst, po);
        plan_key_pack(k, q);
        noise |= plan_key_noise(k);
      }
      if (it == 0) {  // (the hop's first sample is lane 0's first)
        k0 = k;
        q0[0] = __shfl(q[0], 0, HOP_WAVE);
        q0[1] = __shfl(q[1], 0, HOP_WAVE);
      }
      if (i < i1) diff = diff || q[0] != q0[0] || q[1] != q0[1];
    }
    bool mixed = __ballot(diff) != 0;
#pragma unroll
    for (int o = HOP_WAVE / 2; o >= 1; o /= 2) noise |= __shfl_xor(noise, o, HOP_WAVE);
    if (lane == 0) {
      PlanHop &hl = *reinterpret_cast<PlanHop *>(hop_lds);
      hl = PlanHop{};
      const bool ok = plan_hop_inputs(k0, fl, fr, a.uo, a.two_mass != 0, hl);
      hl.mixed = (mixed || !ok) ? 1u : 0u;
      // (compact: the next free slot, claimed by mixed hops only -- the listed hops whose samples
      // share one decision, most of them, need none)
      hl.dense = (a.compact && hl.mixed) ? atomicAdd(a.work + 1, 1u) : 0u;
      hl.noise = noise;  // (every sample's, not only the first's)
    }
    __syncthreads();
    mixed = reinterpret_cast<const PlanHop *>(hop_lds)->mixed != 0;
    const uint32_t slot_e = reinterpret_cast<const PlanHop *>(hop_lds)->dense;
    if (a.compact && (int64_t)slot_e >= a.dense_cap) mixed = false;  // (no room: the host falls back)
    uint64_t *dst = reinterpret_cast<uint64_t *>(a.hops + row * a.hop_stride + slot);
    for (int w = lane; w < HOP_WORDS; w += HOP_WAVE) dst[w] = hop_lds[w];
    if (mixed) {  // the decisions change within the hop: the samples' dense records
      for (int i = i0 + lane; i < i1; i += HOP_WAVE) {
        uint64_t w[PLAN_WORDS];
        plan_sample<true>(fl, fr, (double)i / (double)a.hop, a.uo, a.two_mass != 0, w);
        const int64_t rec = a.compact ? (int64_t)slot_e * a.hop + i : row * a.plan_stride + (h * a.hop + i - a.s_begin);
        ulonglong2 *o = (ulonglong2 *)(a.plan + rec * PLAN_WORDS);
#pragma unroll
        for (int q = 0; q < PLAN_WORDS / 2; ++q) o[q] = make_ulonglong2(w[2 * q], w[2 * q + 1]);
      }
    }
    __syncthreads();  // (the next entry overwrites the LDS frames and record)
  }
}

}  // namespace

hipError_t launch_plan_hops_iv(const PlanArgs &a, hipStream_t st) {
  const int64_t n = a.s_end - a.s_begin;
  if (n <= 0 || a.rows <= 0) return hipSuccess;
  if (!a.hops || a.hop < PLAN_HOP_MIN) return hipErrorInvalidValue;
  if (!a.work) return hipErrorInvalidValue;
  const int64_t slots = plan_hop_slots(a.s_begin, a.s_end, a.hop), n_hops = (int64_t)a.rows * slots;
  hipError_t e = hipMemsetAsync(a.work, 0, 2 * sizeof(uint32_t), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(plan_hop_iv_kernel, dim3((unsigned)((n_hops + HOP_IV_BLOCK - 1) / HOP_IV_BLOCK)),
                     dim3(HOP_IV_BLOCK), 0, st, a, slots);
  return hipGetLastError();
}

hipError_t launch_plan_hops_wave(const PlanArgs &a, hipStream_t st) {
  const int64_t n = a.s_end - a.s_begin;
  if (n <= 0 || a.rows <= 0) return hipSuccess;
  if (!a.hops || a.hop < PLAN_HOP_MIN || !a.work) return hipErrorInvalidValue;
  const int64_t slots = plan_hop_slots(a.s_begin, a.s_end, a.hop), n_hops = (int64_t)a.rows * slots;
  // (a fixed grid: the list's length is on the device; every wave leaves its loop at its end)
  const int64_t waves = n_hops < 2048 ? n_hops : 2048;
  hipLaunchKernelGGL(plan_hop_wave_kernel, dim3((unsigned)waves), dim3(HOP_WAVE), 0, st, a, slots);
  return hipGetLastError();
}

hipError_t launch_plan_hops(const PlanArgs &a, hipStream_t st) {
  const hipError_t e = launch_plan_hops_iv(a, st);
  return e != hipSuccess ? e : launch_plan_hops_wave(a, st);
}

hipError_t launch_plan(const PlanArgs &a, hipStream_t st) {
  const int64_t n = a.s_end - a.s_begin;
  if (n <= 0 || a.rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(plan_kernel, dim3((unsigned)a.rows, (unsigned)((n + PLAN_BLOCK - 1) / PLAN_BLOCK)),
                     dim3(PLAN_BLOCK), 0, st, a);
  return hipGetLastError();
}

// (see preload_tree_kernels, tds_tree.hip)
hipError_t preload_plan_kernels() {
  hipFuncAttributes at;
  hipError_t e = hipFuncGetAttributes(&at, reinterpret_cast<const void *>(plan_kernel));
  if (e == hipSuccess) e = hipFuncGetAttributes(&at, reinterpret_cast<const void *>(plan_hop_iv_kernel));
  if (e == hipSuccess) e = hipFuncGetAttributes(&at, reinterpret_cast<const void *>(plan_hop_wave_kernel));
  return e;
}

}  // namespace afs
