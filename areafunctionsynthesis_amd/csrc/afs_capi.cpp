// afs_capi.cpp -- the C ABI of include/afs.h: contexts, sessions, staging, launches.
//
// Host-side orchestration only; all synthesis arithmetic runs in the HIP kernels.
// There is no CPU fallback: without a usable HIP device afs_create fails with
// AFS_ERR_NO_DEVICE.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "afs_af.h"
#include "afs_lane.h"
#include "afs_audio.h"
#include "afs_ctx.h"
#include "afs_model.h"
#include "afs_tree.h"

static_assert(sizeof(afs_frame) == 1072, "afs_frame layout");

namespace afs {

afs_status fail(afs_ctx *c, afs_status s, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return s;
}

bool is_device_ptr(const void *p) {
  if (!p) return false;
  hipPointerAttribute_t at;
  hipError_t e = hipPointerGetAttributes(&at, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged;
}

// Lanes per utterance of the tree kernel for a batch of B: forced by AFS_LANES_16 / AFS_LANES_64,
// else the voice kernel (64 lanes, one utterance per wave: fewer instructions per sample on the
// chain) while the batch leaves SIMDs idle with 16 lanes per utterance (B <= the GPU's SIMDs), the
// throughput kernel (16 lanes, four utterances per wave) above.
int lanes_for(const afs_ctx *c, int64_t B) {
  if (c->cfg.flags & AFS_LANES_16) return TREE_W;
  if (c->cfg.flags & AFS_LANES_64) return TREE_VOICE_W;
  return B <= c->simds ? TREE_VOICE_W : TREE_W;
}

afs_status ensure(afs_ctx *c, void **buf, size_t *cap, size_t bytes) {
  if (bytes <= *cap) return AFS_OK;
  if (*buf) (void)hipFree(*buf);
  *buf = nullptr;
  *cap = 0;
  HIP_TRY(c, hipMalloc(buf, bytes));
  *cap = bytes;
  return AFS_OK;
}

}  // namespace afs

using afs::ensure;
using afs::fail;
using afs::is_device_ptr;
using afs::lanes_for;

namespace {

int64_t pad64(int64_t b) { return (b + 63) / 64 * 64; }

bool solver_ok(int32_t s) { return s == AFS_SOLVER_CHOLESKY || s == AFS_SOLVER_TREE || s == AFS_SOLVER_SOR; }

// the cooperative kernel (noise-source plans from K5)
bool tree(const afs_ctx *c) { return c->cfg.solver == AFS_SOLVER_TREE; }


// Bytes of noise-source plans one call may hold (afs_ctx::plan_budget: 4 GiB, or
// AFS_PLAN_BUDGET_MB).  Hop mode keeps the hop records of the whole call and the dense records
// of its mixed hops within it (static vowels: 446 MB of records for 8192 utterances x 1 s) and
// runs launches of up to afs_ctx::launch_cap samples; the dense path (hops < 32, or past the
// budget) runs launches of at most plan_budget / (rows * 128 B) samples (4096 at 8192 rows).
// (Round 2 measured one launch per second with 46 GB of dense records no faster than 11
// launches; round 4's compact hop-mode plans make the one launch +0.1..0.5 %,
// profiles/r04h_launch_ab.txt.)
constexpr int64_t PLAN_BUDGET_DEFAULT = (int64_t)4 << 30;
// Hop mode: calls whose dense records fit this many bytes even with every hop listed skip the
// read-back of K5's work-list length (run_chunks).
constexpr int64_t SMALL_CALL_DENSE_BYTES = (int64_t)64 << 20;

// Launch the synthesis of frame transitions 1 .. ntrans (frames[row * fstride + k], k = 0 the
// latched frame) in chunks that keep each kernel well below a second; state is carried
// between launches.  rows: number of distinct frame rows (B, or the target sequences).
// AFS_PROFILE: record an event on the context's stream (a pooled one; recording stops past
// the pool's cap until afs_kernel_times drains it).
hipEvent_t prof_event(afs_ctx *c, hipStream_t st) {
  if (!(c->cfg.flags & AFS_PROFILE)) return nullptr;
  constexpr size_t CAP = 1 << 14;
  if (c->pev_used == c->pev.size()) {
    hipEvent_t e = nullptr;
    if (c->pev.size() >= CAP || hipEventCreate(&e) != hipSuccess) {
      c->timed_overflow = true;
      return nullptr;
    }
    c->pev.push_back(e);
  }
  hipEvent_t e = c->pev[c->pev_used++];
  if (hipEventRecord(e, st) != hipSuccess) return nullptr;
  return e;
}
hipEvent_t prof_event(afs_ctx *c) { return prof_event(c, c->stream); }
void prof_pair(afs_ctx *c, hipEvent_t a, hipEvent_t b, int kind) {
  if (a && b) c->timed.push_back({a, b, kind});
}

// Slot order of the tree kernel for utterances that share trajectories (row[u]: the utterance's
// frame row): the utterances sorted by row, and the sorted list cut into contiguous chunks so that
// the blocks one XCD runs at the same time play as few rows as possible -- each of the 8 XCDs has
// its own L2, and blocks are dealt to them round-robin (block b shares an XCD with b + 8,
// MI355X_MICROARCH.md, workgroup dispatch), in rounds of `conc` blocks (the blocks the GPU holds
// at once).  Entry (block * upb + g) = the utterance of that slot, B for padding slots.
std::vector<int32_t> xcd_order(const std::vector<int32_t> &row, int B, int upb, int conc) {
  constexpr int XCDS = 8;
  std::vector<int32_t> idx((size_t)B);
  for (int u = 0; u < B; ++u) idx[(size_t)u] = u;
  std::stable_sort(idx.begin(), idx.end(), [&](int32_t a, int32_t b) { return row[(size_t)a] < row[(size_t)b]; });
  const int nb = (B + upb - 1) / upb;
  conc = std::max(conc, 1);
  std::vector<int32_t> order((size_t)nb * (size_t)upb, B);
  for (int r0 = 0; r0 < nb; r0 += conc) {  // one round: blocks r0 .. r0 + nr - 1
    const int nr = std::min(conc, nb - r0);
    int chunk = r0;  // (the sorted chunks of this round, XCD by XCD)
    for (int x = 0; x < XCDS; ++x)
      for (int b = r0 + x; b < r0 + nr; b += XCDS, ++chunk)
        for (int g = 0; g < upb; ++g) {
          const int64_t q = (int64_t)chunk * upb + g;
          if (q < B) order[(size_t)b * upb + g] = idx[(size_t)q];
        }
  }
  return order;
}

// A call's slot order for K1 (shape_order): the order (null: the identity), the launch's blocks, and
// whether K1 may run the noise-phase variants (variants_dev: decided on the device, else `variants`).
struct SlotOrder {
  const int32_t *order = nullptr;
  int grid = 0;
  bool variants = true;
  const int32_t *variants_dev = nullptr;
};
// the slot order of a call without one (the voice kernel, sessions, target sequences, small batches)
SlotOrder plain_order(const afs_ctx *c) {
  SlotOrder so;
  so.variants = c->noise_variants != 0;
  return so;
}

afs_status run_chunks(afs_ctx *c, const afs_frame *frames, int64_t fstride, int rows, int ntrans, int hop,
                      double *out, int64_t ostride, void *ws, int32_t *rng, void *lanes, int64_t bp, int B,
                      int width, const int32_t *frame_row, const SlotOrder &so) {
  if (tree(c)) {
    const int64_t S = (int64_t)ntrans * hop;
    const int two = c->cfg.options.glottis_model == AFS_GLOTTIS_TWO_MASS ? 1 : 0;
    const afs::SecRec *uo = c->dev_tab->consts.sec;
    afs_status st;
    // K6's glottal-tone input: section 25's pressure per sample of a launch.  Laid out so that
    // every utterance's row sits at the same position in its 128-byte lines as its output row
    // (stride and base congruent to the output's modulo 16 doubles): K1 stores both through one
    // line-aligned window (tree_kernel.h).
    auto p25_for = [&](int64_t per, int64_t *stride) -> afs_status {
      if (AFS_TONE_K6 != 1) return AFS_OK;  // (the tone filter in K1: no pressures stored)
      *stride = per + ((ostride - per) % 16 + 16) % 16;
      return ensure(c, &c->p25, &c->p25_bytes, ((size_t)B * (size_t)*stride + 32) * sizeof(double));
    };
    auto p25_row0 = [&](int64_t s0) {  // the p25 base for the launch whose outputs start at out + s0
      const int64_t want = (int64_t)((reinterpret_cast<uintptr_t>(out + s0) >> 3) & 15);
      const int64_t have = (int64_t)((reinterpret_cast<uintptr_t>(c->p25) >> 3) & 15);
      return (double *)c->p25 + ((want - have) % 16 + 16) % 16;
    };
    // K1 over samples [s0, s1), then K6 over them (both timed)
    // (skip: the launches of the hop-mode fast path when its compact slots may overflow: they do
    // nothing when K5 claimed more than skip_cap slots)
    auto synth = [&](int64_t s0, int64_t s1, const uint64_t *plan, int64_t plan_stride, const afs::tree::PlanHop *hops,
                     int64_t hop_stride, int64_t p25_stride, const uint32_t *skip = nullptr,
                     int64_t skip_cap = 0) -> afs_status {
      afs::TreeArgs a{c->dev_tab, frames, fstride, frame_row, hop, s0, s1, out + s0, ostride, plan, plan_stride, lanes,
                      (double *)ws, B, c->host_tab.uni, hops, hop_stride, p25_row0(s0), p25_stride, so.order,
                      so.variants ? 1 : 0, so.grid, so.variants_dev, skip, skip_cap};
      {  // the pairs' STAT priority mode by the launch's rounds of workgroups per CU slot (two per CU)
        const int64_t blocks = so.grid > 0 ? so.grid : ((int64_t)B + afs::TREE_UPB - 1) / afs::TREE_UPB;
        const int64_t slots = std::max<int64_t>(1, c->simds / 2), rounds = (blocks + slots - 1) / slots;
        a.stat_prio = c->stat_prio >= 0 ? c->stat_prio : ((width == afs::TREE_W && rounds >= 2) ? 2 : 0);
      }
      hipEvent_t e1 = prof_event(c);
      HIP_TRY(c, afs::launch_tree_synth(a, width, c->stream));
      hipEvent_t e2 = prof_event(c);
      prof_pair(c, e1, e2, 0);
      // K6: the glottal-tone filter and the output stage of the launch's samples
      HIP_TRY(c, afs::launch_tree_output(c->dev_tab, (double *)ws, out + s0, ostride, s1 - s0, B,
                                         AFS_TONE_K6 == 1 ? p25_row0(s0) : nullptr, p25_stride,
                                         c->cfg.options.radiation_from_skin, c->stream, skip, skip_cap));
      prof_pair(c, e2, prof_event(c), 2);
      return AFS_OK;
    };
    // Hop mode (tree solver, hops >= PLAN_HOP_MIN): K5 decides every hop of the call first -- one
    // record per (row, hop), the hops it cannot decide at once listed -- and K5's second stage
    // decides the listed hops sample by sample, writing the dense records of the mixed ones (whose
    // samples differ) into a compact array (one hop-long slot each, claimed from a counter).  K1
    // then runs the call in launches of up to 65536 samples, each hop's words evaluated from its
    // record (or read from its dense slot).  One K1 launch per second of 44.1 kHz audio instead of
    // one per 4096 samples: no state save / restore and launch tail in between (+0.6 %,
    // profiles/r04c_store_launch_ab.txt).  A call whose mixed hops' records would exceed the plan
    // budget falls back to the chunked path.
    const bool hops = !c->plan_dense && hop >= afs::tree::PLAN_HOP_MIN;
    const int64_t call_hops = afs::plan_hop_slots(0, S, hop);
    if (hops && (int64_t)rows * call_hops * (int64_t)sizeof(afs::tree::PlanHop) <= c->plan_budget) {
      const int64_t hstride = call_hops;
      const size_t hbytes = (size_t)rows * (size_t)hstride * sizeof(afs::tree::PlanHop);
      if ((st = ensure(c, &c->hops[0], &c->hops_bytes[0], hbytes)) != AFS_OK) return st;
      if ((st = ensure(c, &c->plan_work[0], &c->plan_work_bytes[0], (size_t)afs::plan_work_bytes(rows, hstride))) != AFS_OK)
        return st;
      afs::tree::PlanHop *hbuf = (afs::tree::PlanHop *)c->hops[0];
      uint32_t *work = (uint32_t *)c->plan_work[0];
      afs::PlanArgs pa{c->dev_tab, frames, fstride, rows, hop, 0, S, nullptr, 0, two, uo, hbuf, hstride, work, true};
      hipEvent_t e0 = prof_event(c);
      HIP_TRY(c, afs::launch_plan_hops_iv(pa, c->stream));
      // Slots for the mixed hops: one for every hop of the call when they fit the budget (small calls:
      // real-time sessions, short batches), else the budget's worth.  No host read-back before K1: the
      // launches are queued at once, guarded by the count of slots K5's second stage claimed (they do
      // nothing if it exceeds the slots); the host then waits for K5 alone -- the launches are already
      // queued behind it, so the device never idles for the host -- and, in the rare call whose mixed
      // hops overflowed the slots, queues the chunked path below (most listed hops are not mixed:
      // near-ties decided alike by every sample; static vowels have none).
      const int64_t slot_bytes = (int64_t)hop * afs::PLAN_RECORD_BYTES;
      const int64_t every = (int64_t)rows * call_hops;
      const bool small = every * slot_bytes <= std::min<int64_t>(c->plan_budget, SMALL_CALL_DENSE_BYTES);
      const int64_t cap = small ? every : std::min<int64_t>(every, std::max<int64_t>(1, c->plan_budget / slot_bytes));
      if ((st = ensure(c, &c->plan, &c->plan_bytes, (size_t)(cap * slot_bytes))) != AFS_OK) return st;
      pa.plan = (uint64_t *)c->plan;
      pa.dense_cap = cap;
      HIP_TRY(c, afs::launch_plan_hops_wave(pa, c->stream));
      const bool guard = cap < every;
      if (guard) {
        HIP_TRY(c, hipMemcpyAsync(c->hcount, work + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipEventRecord(c->ev_k5, c->stream));
      }
      prof_pair(c, e0, prof_event(c), 1);
      const int64_t per = std::min<int64_t>(S, c->launch_cap);
      int64_t p25_stride = 0;
      if ((st = p25_for(per, &p25_stride)) != AFS_OK) return st;
      for (int64_t s0 = 0; s0 < S; s0 += per) {
        const int64_t s1 = std::min(S, s0 + per);
        // (K1 indexes the records from the launch's first hop)
        if ((st = synth(s0, s1, (const uint64_t *)c->plan, 0, hbuf + s0 / hop, hstride, p25_stride,
                        guard ? work + 1 : nullptr, cap)) != AFS_OK)
          return st;
      }
      if (!guard) return AFS_OK;
      HIP_TRY(c, hipEventSynchronize(c->ev_k5));
      if ((int64_t)(uint32_t)*c->hcount <= cap) return AFS_OK;
      // (overflow: the guarded launches did nothing, the state is still the call's initial state)
    }
    // Chunked path: launches of `per` samples, each K5 (the chunk's plans: dense records, or in
    // hop mode the chunk's hop records with sample-indexed dense records) and then K1.  With
    // AFS_PLAN_OVERLAP=1 in the environment (afs_ctx::overlap), K5 of chunk k + 1 runs on the plan
    // stream beside K1 of chunk k instead: two plan buffers, K5 of chunk k + 1 waits until K1 of
    // chunk k - 1 has read that buffer, K1 of chunk k waits for its plans.  K5 (80 VGPRs, 4 KB of
    // LDS per block) fits beside K1's wave, but the measured gain (+1.4 %) came with runs where K1
    // slowed by 9 % beside it, so the default is sequential.
    // Dense records: `per` samples per row.  Hop mode: the compact dense records of the chunk's
    // listed hops, slot e of the work list holding `hop` records, and every hop the chunk spans may
    // be listed -- rows x hstride slots of hop records, hstride = the chunk's hop slots + 1 (a chunk
    // may start inside a hop).  Chunks of whole hops are sized so that this worst case fits the
    // budget (at least one hop per chunk: past that the budget is exceeded, not the buffer).
    int64_t per = std::min<int64_t>(S, c->launch_cap);
    if (hops) {
      const int64_t slots_fit = c->plan_budget / ((int64_t)rows * hop * afs::PLAN_RECORD_BYTES) - 1;
      per = std::min<int64_t>(per, std::max<int64_t>(1, slots_fit) * hop);
    } else {
      per = std::min<int64_t>(per, c->plan_budget / ((int64_t)rows * afs::PLAN_RECORD_BYTES));
    }
    per = std::max<int64_t>(1, per);
    const int64_t nch = (S + per - 1) / per;
    const int64_t hstride = afs::plan_hop_slots(0, per, hop) + 1;
    const size_t pbytes = (size_t)rows * (size_t)(hops ? hstride * hop : per) * afs::PLAN_RECORD_BYTES;
    if ((st = ensure(c, &c->plan, &c->plan_bytes, pbytes)) != AFS_OK) return st;
    const bool ov = c->overlap && nch > 1;
    if (ov && (st = ensure(c, &c->plan2, &c->plan2_bytes, pbytes)) != AFS_OK) return st;
    void *buf[2] = {c->plan, ov ? c->plan2 : c->plan};
    afs::tree::PlanHop *hbuf[2] = {nullptr, nullptr};
    if (hops) {
      const size_t hbytes = (size_t)rows * (size_t)hstride * sizeof(afs::tree::PlanHop);
      const size_t wbytes = (size_t)afs::plan_work_bytes(rows, hstride);
      for (int q = 0; q < (ov ? 2 : 1); ++q) {
        if ((st = ensure(c, &c->hops[q], &c->hops_bytes[q], hbytes)) != AFS_OK) return st;
        if ((st = ensure(c, &c->plan_work[q], &c->plan_work_bytes[q], wbytes)) != AFS_OK) return st;
      }
      hbuf[0] = (afs::tree::PlanHop *)c->hops[0];
      hbuf[1] = (afs::tree::PlanHop *)c->hops[ov ? 1 : 0];
    }
    int64_t p25_stride = 0;
    if ((st = p25_for(per, &p25_stride)) != AFS_OK) return st;
    hipStream_t ps = ov ? c->plan_stream : c->stream;
    auto plan_chunk = [&](int64_t k) -> afs_status {
      const int64_t s0 = k * per, s1 = std::min(S, s0 + per);
      afs::PlanArgs pa{c->dev_tab, frames, fstride, rows, hop, s0, s1, (uint64_t *)buf[k & 1], per, two, uo,
                       hbuf[k & 1], hstride, hops ? (uint32_t *)c->plan_work[ov ? (k & 1) : 0] : nullptr, hops,
                       (int64_t)rows * hstride};  // (hop mode: a slot for every hop of the chunk)
      hipEvent_t e0 = prof_event(c, ps);
      HIP_TRY(c, hops ? afs::launch_plan_hops(pa, ps) : afs::launch_plan(pa, ps));
      prof_pair(c, e0, prof_event(c, ps), 1);
      if (ov) HIP_TRY(c, hipEventRecord(c->ev_plan[k & 1], ps));
      return AFS_OK;
    };
    if (ov) {  // (the frames may have been uploaded on the context's stream just before)
      HIP_TRY(c, hipEventRecord(c->ev_go, c->stream));
      HIP_TRY(c, hipStreamWaitEvent(ps, c->ev_go, 0));
      if ((st = plan_chunk(0)) != AFS_OK) return st;
    }
    for (int64_t k = 0; k < nch; ++k) {
      if (!ov) {
        if ((st = plan_chunk(k)) != AFS_OK) return st;
      } else {
        if (k + 1 < nch) {
          if (k >= 1) HIP_TRY(c, hipStreamWaitEvent(ps, c->ev_free[(k + 1) & 1], 0));
          if ((st = plan_chunk(k + 1)) != AFS_OK) return st;
        }
        HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_plan[k & 1], 0));
      }
      const int64_t s0 = k * per, s1 = std::min(S, s0 + per);
      if ((st = synth(s0, s1, (const uint64_t *)buf[k & 1], per, hbuf[k & 1], hstride, p25_stride)) != AFS_OK) return st;
      if (ov) HIP_TRY(c, hipEventRecord(c->ev_free[k & 1], c->stream));
    }
    return AFS_OK;
  }
  const int per = (int)std::max<int64_t>(1, 8192 / std::max(1, hop));
  for (int k = 1; k <= ntrans; k += per) {
    const int ke = std::min(ntrans + 1, k + per);
    double *o = out + (int64_t)(k - 1) * hop;
    afs::LaneArgs a{c->dev_tab, frames, fstride, frame_row, k, ke, hop, o, ostride, (double *)ws, rng, bp, B,
                    c->cfg.solver == AFS_SOLVER_SOR ? 1 : 0};
    hipEvent_t e0 = prof_event(c);
    HIP_TRY(c, afs::launch_lane_synth(a, c->stream));
    prof_pair(c, e0, prof_event(c), 0);
  }
  return AFS_OK;
}

// bytes of the state buffers for B utterances
size_t ws_bytes_for(const afs_ctx *c, int64_t bp) {
  if (tree(c)) return (size_t)bp * afs::tree_lds_doubles() * sizeof(double);
  return (size_t)(afs::lane_ws_rows(c->host_tab) * bp) * sizeof(double);
}
size_t lanes_bytes_for(const afs_ctx *c, int64_t bp, int width) {
  return tree(c) ? (size_t)bp * (size_t)width * (size_t)afs::tree_lane_bytes(width) : 0;
}

afs_status reset_state(afs_ctx *c, void *ws, int32_t *rng, void *lanes, int64_t bp, int B, const uint32_t *seeds_dev,
                       int width) {
  if (tree(c))
    HIP_TRY(c, afs::launch_tree_reset(lanes, (double *)ws, B, seeds_dev, width, c->stream));
  else
    HIP_TRY(c, afs::launch_lane_reset((double *)ws, rng, bp, B, seeds_dev, c->stream));
  return AFS_OK;
}

// Per-utterance non-finite flags (into `flags`, a host or device array of B bytes, or nowhere)
// and their count (into the pinned c->hcount, read after the stream synchronises).  *host_sync
// is set when the flags go to host memory (the call must synchronise before returning).
afs_status nonfinite_report(afs_ctx *c, void *ws, int64_t bp, int B, uint8_t *flags, bool want_count,
                            bool *host_sync) {
  *host_sync = false;
  if (!flags && !want_count) return AFS_OK;
  uint8_t *dflags = flags;
  if (flags && !is_device_ptr(flags)) {
    afs_status s = ensure(c, &c->stage_nf, &c->stage_nf_bytes, (size_t)B);
    if (s != AFS_OK) return s;
    dflags = (uint8_t *)c->stage_nf;
    *host_sync = true;
  }
  HIP_TRY(c, hipMemsetAsync(c->dcount, 0, sizeof(int32_t), c->stream));
  if (tree(c))
    HIP_TRY(c, afs::launch_tree_nonfinite((const double *)ws, B, c->dcount, dflags, c->stream));
  else
    HIP_TRY(c, afs::launch_lane_nonfinite((const double *)ws, bp, B, c->dcount, dflags, c->stream));
  if (*host_sync) HIP_TRY(c, hipMemcpyAsync(flags, dflags, (size_t)B, hipMemcpyDeviceToHost, c->stream));
  if (want_count) HIP_TRY(c, hipMemcpyAsync(c->hcount, c->dcount, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  return AFS_OK;
}

afs_status draws_of(afs_ctx *c, const void *ws, int B, int64_t *draws) {
  if (!tree(c)) return fail(c, AFS_ERR_UNSUPPORTED, "rand() call counts are kept by the tree solver only");
  int64_t *d = draws;
  void *tmp = nullptr;
  if (!is_device_ptr(draws)) {
    HIP_TRY(c, hipMalloc(&tmp, (size_t)B * sizeof(int64_t)));
    d = (int64_t *)tmp;
  }
  hipError_t e = afs::launch_tree_draws((const double *)ws, B, d, c->stream);
  if (e == hipSuccess && tmp) e = hipMemcpyAsync(draws, d, (size_t)B * sizeof(int64_t), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (tmp) (void)hipFree(tmp);
  if (e != hipSuccess) return fail(c, AFS_ERR_HIP, "afs_rng_draws: %s", hipGetErrorString(e));
  return AFS_OK;
}

}  // namespace

extern "C" {

int32_t afs_abi_version(void) { return AFS_ABI_VERSION; }

void afs_config_default(afs_config *cfg) {
  if (!cfg) return;
  std::memset(cfg, 0, sizeof *cfg);
  cfg->sampling_rate_hz = 22050.0;
  cfg->precision = AFS_FP64;
  cfg->solver = AFS_SOLVER_TREE;  // (the fastest kernel: DESIGN.md 4)
  cfg->device = 0;
  cfg->flags = 0;
  cfg->options = afs::default_options();
}

const char *afs_status_string(afs_status s) {
  switch (s) {
    case AFS_OK: return "ok";
    case AFS_ERR_INVALID_ARGUMENT: return "invalid argument";
    case AFS_ERR_NO_DEVICE: return "no HIP device";
    case AFS_ERR_HIP: return "HIP runtime error";
    case AFS_ERR_OUT_OF_MEMORY: return "out of device memory";
    case AFS_ERR_UNSUPPORTED: return "unsupported configuration";
  }
  return "unknown status";
}

afs_status afs_create(afs_ctx **out, const afs_config *cfg) {
  if (!out) return AFS_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  afs_config c;
  if (cfg) c = *cfg; else afs_config_default(&c);
  if (!(c.sampling_rate_hz > 0.0) || c.precision != AFS_FP64 || !solver_ok(c.solver) ||
      ((c.flags & AFS_LANES_16) && (c.flags & AFS_LANES_64)))
    return AFS_ERR_INVALID_ARGUMENT;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
    (void)hipGetLastError();
    return AFS_ERR_NO_DEVICE;
  }
  if (c.device < 0 || c.device >= n) return AFS_ERR_NO_DEVICE;
  if (hipSetDevice(c.device) != hipSuccess) return AFS_ERR_NO_DEVICE;
  afs_ctx *ctx = new afs_ctx();
  ctx->cfg = c;
  {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c.device) != hipSuccess || cus <= 0) cus = 256;
    ctx->simds = 4 * cus;  // (4 SIMDs per CU on CDNA)
  }
  afs::build_tables(&ctx->host_tab, c.sampling_rate_hz, c.options);
  if (ctx->host_tab.n_rounds <= 0) { afs_destroy(ctx); return AFS_ERR_UNSUPPORTED; }
  afs_status st = AFS_OK;
  auto bail = [&](afs_status s) { afs_destroy(ctx); return s; };
  if (hipMalloc((void **)&ctx->dev_tab, sizeof(afs::Tables)) != hipSuccess) return bail(AFS_ERR_OUT_OF_MEMORY);
  if (hipMemcpy(ctx->dev_tab, &ctx->host_tab, sizeof(afs::Tables), hipMemcpyHostToDevice) != hipSuccess)
    return bail(AFS_ERR_HIP);
  if (hipMalloc((void **)&ctx->dcount, sizeof(int32_t)) != hipSuccess) return bail(AFS_ERR_OUT_OF_MEMORY);
  if (hipHostMalloc((void **)&ctx->hcount, sizeof(int32_t), hipHostMallocDefault) != hipSuccess)
    return bail(AFS_ERR_OUT_OF_MEMORY);
  *ctx->hcount = 0;
  if (hipEventCreate(&ctx->ev0) != hipSuccess || hipEventCreate(&ctx->ev1) != hipSuccess) return bail(AFS_ERR_HIP);
  // the code objects of the kernels a synthesis call launches, loaded now rather than at their
  // first launch (which cost a real-time caller's first buffer ~35 ms)
  if (afs::preload_tree_kernels() != hipSuccess || afs::preload_plan_kernels() != hipSuccess ||
      afs::preload_audio_kernels() != hipSuccess)
    return bail(AFS_ERR_HIP);
  if (const char *e = std::getenv("AFS_PLAN_OVERLAP")) ctx->overlap = std::atoi(e) != 0;
  if (const char *e = std::getenv("AFS_PLAN_DENSE")) ctx->plan_dense = std::atoi(e) != 0;
  if (const char *e = std::getenv("AFS_XCD_ORDER")) ctx->xcd_order = std::atoi(e) != 0;
  if (const char *e = std::getenv("AFS_SHAPE_ORDER")) ctx->shape_order = std::atoi(e) != 0;
  if (const char *e = std::getenv("AFS_NOISE_VARIANTS")) ctx->noise_variants = std::atoi(e);
  if (const char *e = std::getenv("AFS_CLASS_ORDER")) ctx->class_order = std::atoi(e);
  if (const char *e = std::getenv("AFS_STAT_PRIO")) ctx->stat_prio = std::atoi(e);
  if (const char *e = std::getenv("AFS_LAUNCH_SAMPLES")) {  // (A/B and latency studies: samples per K1 launch)
    const long long v = std::atoll(e);
    if (v > 0) ctx->launch_cap = std::min<int64_t>(v, 65536);
  }
  if (hipStreamCreateWithFlags(&ctx->plan_stream, hipStreamNonBlocking) != hipSuccess) return bail(AFS_ERR_HIP);
  for (hipEvent_t *e : {&ctx->ev_go, &ctx->ev_plan[0], &ctx->ev_plan[1], &ctx->ev_free[0], &ctx->ev_free[1], &ctx->ev_k5})
    if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) return bail(AFS_ERR_HIP);
  {
    ctx->plan_budget = PLAN_BUDGET_DEFAULT;
    if (const char *e = std::getenv("AFS_PLAN_BUDGET_MB")) {
      const long long mb = std::atoll(e);
      if (mb > 0) ctx->plan_budget = (int64_t)mb << 20;
    }
  }
  (void)st;
  *out = ctx;
  return AFS_OK;
}

void afs_destroy(afs_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->cfg.device);
  if (c->dev_tab) (void)hipFree(c->dev_tab);
  if (c->ws) (void)hipFree(c->ws);
  if (c->rng) (void)hipFree(c->rng);
  if (c->tree_lanes) (void)hipFree(c->tree_lanes);
  if (c->stage_in) (void)hipFree(c->stage_in);
  if (c->stage_out) (void)hipFree(c->stage_out);
  if (c->stage_seeds) (void)hipFree(c->stage_seeds);
  if (c->tgt) (void)hipFree(c->tgt);
  if (c->keys) (void)hipFree(c->keys);
  if (c->order_buf) (void)hipFree(c->order_buf);
  if (c->sort_tmp) (void)hipFree(c->sort_tmp);
  if (c->plan_stream) (void)hipStreamSynchronize(c->plan_stream);
  if (c->plan) (void)hipFree(c->plan);
  if (c->plan2) (void)hipFree(c->plan2);
  for (void *h : c->hops)
    if (h) (void)hipFree(h);
  for (void *w : c->plan_work)
    if (w) (void)hipFree(w);
  if (c->p25) (void)hipFree(c->p25);
  if (c->plan_stream) (void)hipStreamDestroy(c->plan_stream);
  for (hipEvent_t e : {c->ev_go, c->ev_plan[0], c->ev_plan[1], c->ev_free[0], c->ev_free[1], c->ev_k5})
    if (e) (void)hipEventDestroy(e);
  if (c->stage_nf) (void)hipFree(c->stage_nf);
  if (c->dcount) (void)hipFree(c->dcount);
  if (c->hcount) (void)hipHostFree(c->hcount);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  for (hipEvent_t e : c->pev) (void)hipEventDestroy(e);
  for (void *p : {c->m_out, c->m_pcm, c->m_nf, c->m_root})
    if (p) (void)hipFree(p);
  delete c;
}

const char *afs_last_error(const afs_ctx *c) { return c ? c->err.c_str() : "null context"; }

afs_status afs_set_stream(afs_ctx *c, void *s) {
  if (!c) return AFS_ERR_INVALID_ARGUMENT;
  c->stream = (hipStream_t)s;
  return AFS_OK;
}

afs_status afs_synchronize(afs_ctx *c) {
  if (!c) return AFS_ERR_INVALID_ARGUMENT;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return AFS_OK;
}

}  // extern "C"

// Slot order of the 16-lane tree kernel for a batch of independent utterances: sorted by the shape
// key of their first frame (how narrow the tube is and where: launch_utterance_keys), so that the
// four utterances of a wave -- which run in lockstep and pay for the union of their branches
// (noise sources, the cutoff filter's exponential, mixed hops) -- and the blocks of a compute unit
// play alike shapes, the heaviest (narrowest constrictions) first.  Each utterance's audio is the
// same in any slot.  Config-4 shard: +2.7 % static vowels, +1.4 % fricatives against the call order
// (profiles/r04s_shape_order_ab.txt, r04v_shape_key_ab.txt).  Off for the voice kernel (one
// utterance per wave), batches of one block and AFS_SHAPE_ORDER=0.
//
// All on the device, with no host wait (the call's K1 is queued behind it while the previous call's
// K1 still runs): the key kernel, the variant rule and a stable radix sort of (key, utterance)
// (af_kernels.hip launch_slot_order).  The rule: the noise-phase variants pay when most waves are
// light, or when every SIMD runs many waves: at 8192 static vowels (61 % light, two waves per SIMD)
// +2.3 %, at 8192 fricatives (28 % light) -3 % -- the full-phase waves lose more to the light ones'
// copies of the kernel body in their CUs' instruction caches than the light ones gain -- but at 65536
// fricatives (16 waves per SIMD, the classes in long runs of the slot order) +0.7 %, at 32768 (8 per
// SIMD) +0.05 % (profiles/r05i_fricatives_variants_ab.txt, r05k_variant_rule_ab.txt,
// r05r_variant_rule_ab.txt).  Without them the class is left out of the sort (the class key alone
// measured -0.6 %, r05f_variant_order_ab.txt).  (AFS_CLASS_ORDER=3, an A/B study, deals the blocks to
// the XCDs on the host.)
static afs_status shape_order(afs_ctx *c, const afs_frame *dframes, int64_t fstride, int B, int width, SlotOrder *so) {
  *so = plain_order(c);
  const int upb = afs::TREE_UPB;
  if (!tree(c) || !c->shape_order || width == afs::TREE_VOICE_W || B <= upb) return AFS_OK;
  const int nb = (B + upb - 1) / upb;
  const bool by_xcd = c->class_order == 3 && c->noise_variants != 0;
  afs_status s;
  // keys[B], sorted keys[B], indices[B], the variant flag
  const size_t kb = (size_t)B * (2 * sizeof(uint64_t) + sizeof(int32_t)) + 16;
  if ((s = ensure(c, &c->keys, &c->keys_bytes, kb)) != AFS_OK) return s;
  uint64_t *dkeys = (uint64_t *)c->keys;
  HIP_TRY(c, afs::launch_utterance_keys(dframes, fstride, B, dkeys, by_xcd ? 1 : (c->class_order == 3 ? 0 : c->class_order),
                                        c->stream));
  if (!by_xcd) {
    uint64_t *dsorted = dkeys + B;
    int32_t *didx = (int32_t *)(dsorted + B);
    int32_t *dvar = didx + B;
    const int shift = c->class_order == 1 ? 48 : c->class_order == 2 ? 40 : -1;
    const int64_t waves_per_simd = (int64_t)B / ((int64_t)(64 / afs::TREE_W) * std::max(1, c->simds));
    const int mode = c->noise_variants == 0 ? 0 : c->noise_variants == 1 ? 1 : 2;
    if ((s = ensure(c, &c->order_buf, &c->order_bytes, (size_t)nb * upb * sizeof(int32_t))) != AFS_OK) return s;
    size_t tb = 0;
    HIP_TRY(c, afs::launch_slot_order(dkeys, dsorted, didx, B, shift, mode, waves_per_simd >= 16, dvar,
                                      (int32_t *)c->order_buf, nb * upb, nullptr, &tb, c->stream));
    if ((s = ensure(c, &c->sort_tmp, &c->sort_tmp_bytes, tb + 256)) != AFS_OK) return s;
    tb = c->sort_tmp_bytes;
    HIP_TRY(c, afs::launch_slot_order(dkeys, dsorted, didx, B, shift, mode, waves_per_simd >= 16, dvar,
                                      (int32_t *)c->order_buf, nb * upb, c->sort_tmp, &tb, c->stream));
    so->order = (const int32_t *)c->order_buf;
    so->grid = nb;
    so->variants_dev = dvar;
    return AFS_OK;
  }
  c->hkeys.resize((size_t)B);
  HIP_TRY(c, hipMemcpyAsync(c->hkeys.data(), dkeys, (size_t)B * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  std::vector<int32_t> idx((size_t)B);
  for (int u = 0; u < B; ++u) idx[(size_t)u] = u;
  std::stable_sort(idx.begin(), idx.end(),
                   [&](int32_t a, int32_t b) { return c->hkeys[(size_t)a] < c->hkeys[(size_t)b]; });
  int nblocks = nb;
  {
    // The blocks of the class-major order (the full noise phases first) dealt to the 8 XCDs in
    // contiguous runs of equal expected cost, so that the blocks one XCD runs -- whose waves share
    // its CUs' instruction caches -- run one noise-phase variant (at most one change per XCD): a
    // CU pair holds about one copy of the kernel body, and waves of different variants on it
    // slowed each other (profiles/r05i_fricatives_variants_ab.txt).  Blocks are dealt to XCDs
    // round-robin (block b runs on XCD b % 8, MI355X_MICROARCH.md), so run x occupies grid
    // blocks x, x + 8, ...; the shorter runs end in empty blocks, which exit at once.  Expected
    // cost of a block: that of its heaviest utterance's variant, from the ceilings measured with
    // every wave in one variant (profiles/r05b_noise_variant_ceiling_ab.txt).
    constexpr int XCDS = 8;
    static const double cost[4] = {1.0, 0.976, 0.954, 0.885};  // NZ_FULL, NZ_T1ALL, NZ_TONGUE1, NZ_GLOTTIS
    std::vector<double> bc((size_t)nb, 0.0);
    double total = 0.0;
    for (int b = 0; b < nb; ++b) {
      double w = 0.0;
      for (int g = 0; g < upb && b * upb + g < B; ++g)
        w = std::max(w, cost[(c->hkeys[(size_t)idx[(size_t)(b * upb + g)]] >> 48) & 3]);
      bc[(size_t)b] = w;
      total += w;
    }
    std::vector<int> first(XCDS + 1, nb);
    first[0] = 0;
    double acc = 0.0;
    int x = 1;
    for (int b = 0; b < nb && x < XCDS; ++b) {
      acc += bc[(size_t)b];
      if (acc >= total * x / XCDS) first[(size_t)x++] = b + 1;
    }
    for (; x < XCDS; ++x) first[(size_t)x] = nb;
    int len = 0;
    for (int q = 0; q < XCDS; ++q) len = std::max(len, first[(size_t)q + 1] - first[(size_t)q]);
    nblocks = XCDS * len;
    c->horder.assign((size_t)nblocks * upb, B);
    for (int q = 0; q < XCDS; ++q)
      for (int b = first[(size_t)q]; b < first[(size_t)q + 1]; ++b) {
        const int slot = (q + XCDS * (b - first[(size_t)q])) * upb;
        for (int g = 0; g < upb && b * upb + g < B; ++g) c->horder[(size_t)(slot + g)] = idx[(size_t)(b * upb + g)];
      }
  }
  const size_t obytes = c->horder.size() * sizeof(int32_t);
  if ((s = ensure(c, &c->order_buf, &c->order_bytes, obytes)) != AFS_OK) return s;
  HIP_TRY(c, hipMemcpyAsync(c->order_buf, c->horder.data(), obytes, hipMemcpyHostToDevice, c->stream));
  so->order = (const int32_t *)c->order_buf;
  so->grid = nblocks;
  so->variants = true;
  return AFS_OK;
}

// afs_synthesize; force_async: leave the stream running unless a host buffer needs a wait
static afs_status synth_core(afs_ctx *c, const afs_frame *frames, const uint32_t *seeds, int32_t B, int32_t F,
                             int32_t hop, double *out, uint8_t *nonfinite, afs_report *rep, bool force_async,
                             int lanes = 0) {
  if (!frames || !out || B <= 0 || F < 2 || hop < 1)
    return fail(c, AFS_ERR_INVALID_ARGUMENT, "afs_synthesize: need frames, out, batch>0, num_frames>=2, hop>=1");
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  const int64_t T = (int64_t)(F - 1) * hop;
  const int64_t bp = pad64(B);
  afs_status s;
  // inputs
  const afs_frame *dframes = frames;
  if (!is_device_ptr(frames)) {
    size_t bytes = (size_t)B * F * sizeof(afs_frame);
    if ((s = ensure(c, &c->stage_in, &c->stage_in_bytes, bytes)) != AFS_OK) return s;
    HIP_TRY(c, hipMemcpyAsync(c->stage_in, frames, bytes, hipMemcpyHostToDevice, c->stream));
    dframes = (const afs_frame *)c->stage_in;
  }
  const uint32_t *dseeds = seeds;
  if (seeds && !is_device_ptr(seeds)) {
    if ((s = ensure(c, &c->stage_seeds, &c->stage_seeds_bytes, (size_t)B * 4)) != AFS_OK) return s;
    HIP_TRY(c, hipMemcpyAsync(c->stage_seeds, seeds, (size_t)B * 4, hipMemcpyHostToDevice, c->stream));
    dseeds = (const uint32_t *)c->stage_seeds;
  }
  double *dout = out;
  const bool host_out = !is_device_ptr(out);
  if (host_out) {
    if ((s = ensure(c, &c->stage_out, &c->stage_out_bytes, (size_t)B * T * sizeof(double))) != AFS_OK) return s;
    dout = (double *)c->stage_out;
  }
  // state
  const int width = lanes > 0 ? lanes : lanes_for(c, B);
  if ((s = ensure(c, &c->ws, &c->ws_bytes, ws_bytes_for(c, bp))) != AFS_OK) return s;
  if ((s = ensure(c, (void **)&c->rng, &c->rng_bytes, (size_t)(32 * bp) * sizeof(int32_t))) != AFS_OK) return s;
  if (tree(c) && (s = ensure(c, &c->tree_lanes, &c->tree_lanes_bytes, lanes_bytes_for(c, bp, width))) != AFS_OK)
    return s;
  if ((s = reset_state(c, c->ws, c->rng, c->tree_lanes, bp, B, dseeds, width)) != AFS_OK) return s;
  HIP_TRY(c, hipEventRecord(c->ev0, c->stream));
  SlotOrder so;
  if ((s = shape_order(c, dframes, F, B, width, &so)) != AFS_OK) return s;
  if ((s = run_chunks(c, dframes, F, B, F - 1, hop, dout, T, c->ws, c->rng, c->tree_lanes, bp, B, width, nullptr,
                      so)) != AFS_OK)
    return s;
  HIP_TRY(c, hipEventRecord(c->ev1, c->stream));
  c->last_B = B;
  bool nf_sync = false;
  if ((s = nonfinite_report(c, c->ws, bp, B, nonfinite, rep != nullptr, &nf_sync)) != AFS_OK) return s;
  if (host_out) HIP_TRY(c, hipMemcpyAsync(out, dout, (size_t)B * T * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  const bool sync = !(force_async || (c->cfg.flags & AFS_ASYNC)) || host_out || rep || nf_sync;
  if (sync) HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (rep) {
    float ms = 0.f;
    HIP_TRY(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
    rep->device_ms = ms;
    rep->samples = (int64_t)B * T;
    rep->nonfinite_utterances = *c->hcount;
    rep->kernel = c->cfg.solver;
  }
  return AFS_OK;
}

afs_status afs::synthesize_async(afs_ctx *c, const afs_frame *frames, const uint32_t *seeds, int32_t B, int32_t F,
                                 int32_t hop, double *out, uint8_t *nonfinite, int lanes) {
  if (lanes != 0 && lanes != afs::TREE_W && lanes != afs::TREE_VOICE_W)
    return fail(c, AFS_ERR_INVALID_ARGUMENT, "synthesize: %d lanes per utterance", lanes);
  return synth_core(c, frames, seeds, B, F, hop, out, nonfinite, nullptr, true, lanes);
}

extern "C" {

afs_status afs_synthesize(afs_ctx *c, const afs_frame *frames, const uint32_t *seeds, int32_t B,
                          int32_t F, int32_t hop, double *out, uint8_t *nonfinite, afs_report *rep) {
  if (!c) return AFS_ERR_INVALID_ARGUMENT;
  if (!frames || !out || B <= 0 || F < 2 || hop < 1)
    return fail(c, AFS_ERR_INVALID_ARGUMENT, "afs_synthesize: need frames, out, batch>0, num_frames>=2, hop>=1");
  return synth_core(c, frames, seeds, B, F, hop, out, nonfinite, rep, false);
}

int32_t afs_lanes_per_utterance(const afs_ctx *c, int32_t batch) {
  if (!c || c->cfg.solver != AFS_SOLVER_TREE || batch <= 0) return 1;
  return lanes_for(c, batch);
}

const char *afs_synthesis_kernel(const afs_ctx *c, int32_t batch) {
  if (!c || c->cfg.solver != AFS_SOLVER_TREE) return "lane_synth_kernel";
  const int lanes = afs_lanes_per_utterance(c, batch);
  if (AFS_PAIR && lanes == afs::TREE_W) return "tree_pair_kernel";
  if (AFS_PAIR && lanes == afs::TREE_VOICE_W && batch <= afs::TREE_PAIR64_MAX) return "tree_pair64_kernel";
  return "tree_synth_kernel";
}

afs_status afs_kernel_times_ex(afs_ctx *c, afs_kernel_timing *t) {
  if (!c || !t) return AFS_ERR_INVALID_ARGUMENT;
  if (!(c->cfg.flags & AFS_PROFILE)) return fail(c, AFS_ERR_INVALID_ARGUMENT, "afs_kernel_times: AFS_PROFILE is off");
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  double ms[3] = {0.0, 0.0, 0.0};
  int32_t n[3] = {0, 0, 0};
  for (const auto &e : c->timed) {
    float x = 0.f;
    HIP_TRY(c, hipEventElapsedTime(&x, e.a, e.b));
    ms[e.kind] += x;
    ++n[e.kind];
  }
  const bool overflow = c->timed_overflow;
  c->timed.clear();
  c->pev_used = 0;
  c->timed_overflow = false;
  t->synth_ms = ms[0];
  t->synth_launches = n[0];
  t->plan_ms = ms[1];
  t->plan_launches = n[1];
  t->output_ms = ms[2];
  t->output_launches = n[2];
  if (overflow) return fail(c, AFS_ERR_UNSUPPORTED, "afs_kernel_times: more launches than the event pool holds");
  return AFS_OK;
}

afs_status afs_kernel_times(afs_ctx *c, double *synth_ms, int32_t *synth_launches, double *plan_ms,
                            int32_t *plan_launches) {
  afs_kernel_timing t{};
  const afs_status s = afs_kernel_times_ex(c, &t);
  if (synth_ms) *synth_ms = t.synth_ms;
  if (synth_launches) *synth_launches = t.synth_launches;
  if (plan_ms) *plan_ms = t.plan_ms;
  if (plan_launches) *plan_launches = t.plan_launches;
  return s;
}

afs_status afs_rng_draws(afs_ctx *c, int32_t B, int64_t *draws) {
  if (!c) return AFS_ERR_INVALID_ARGUMENT;
  if (!draws || B <= 0 || B != c->last_B || !c->ws)
    return fail(c, AFS_ERR_INVALID_ARGUMENT, "afs_rng_draws: need draws[B] with B = the last call's batch");
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  return draws_of(c, c->ws, B, draws);
}

afs_status afs_noise_plans(afs_ctx *c, const afs_frame *frames, int32_t rows, int32_t F, int32_t hop, int64_t s0,
                           int64_t s1, uint64_t *plans) {
  static_assert(AFS_PLAN_WORDS * 8 == afs::PLAN_RECORD_BYTES, "afs.h / tree_plan.h record size");
  if (!c) return AFS_ERR_INVALID_ARGUMENT;
  if (!tree(c)) return fail(c, AFS_ERR_UNSUPPORTED, "afs_noise_plans: tree solver only");
  if (!frames || !plans || rows <= 0 || F < 2 || hop < 1 || s0 < 0 || s1 <= s0 || s1 > (int64_t)(F - 1) * hop)
    return fail(c, AFS_ERR_INVALID_ARGUMENT, "afs_noise_plans: need frames, plans, rows>0, num_frames>=2, hop>=1, "
                                             "0 <= s_begin < s_end <= (num_frames-1)*hop");
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  afs_status s;
  const afs_frame *dframes = frames;
  if (!is_device_ptr(frames)) {
    const size_t bytes = (size_t)rows * F * sizeof(afs_frame);
    if ((s = ensure(c, &c->stage_in, &c->stage_in_bytes, bytes)) != AFS_OK) return s;
    HIP_TRY(c, hipMemcpyAsync(c->stage_in, frames, bytes, hipMemcpyHostToDevice, c->stream));
    dframes = (const afs_frame *)c->stage_in;
  }
  const int64_t n = s1 - s0;
  const size_t bytes = (size_t)rows * (size_t)n * afs::PLAN_RECORD_BYTES;
  uint64_t *dplans = plans;
  const bool host_out = !is_device_ptr(plans);
  if (host_out) {
    if ((s = ensure(c, &c->plan, &c->plan_bytes, bytes)) != AFS_OK) return s;
    dplans = (uint64_t *)c->plan;
  }
  afs::PlanArgs pa{c->dev_tab, dframes, F, rows, hop, s0, s1, dplans, n,
                   c->cfg.options.glottis_model == AFS_GLOTTIS_TWO_MASS ? 1 : 0,
                   c->dev_tab->consts.sec};
  HIP_TRY(c, afs::launch_plan(pa, c->stream));
  if (host_out) HIP_TRY(c, hipMemcpyAsync(plans, dplans, bytes, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return AFS_OK;
}

afs_status afs_noise_plan_hops(afs_ctx *c, const afs_frame *frames, int32_t rows, int32_t F, int32_t hop, int64_t s0,
                               int64_t s1, uint8_t *hops, uint64_t *plans) {
  static_assert(AFS_PLAN_HOP_BYTES == sizeof(afs::tree::PlanHop), "afs.h / tree_plan.h hop record size");
  static_assert(AFS_PLAN_HOP_MIN == afs::tree::PLAN_HOP_MIN, "afs.h / tree_plan.h hop mode threshold");
  if (!c) return AFS_ERR_INVALID_ARGUMENT;
  if (c->cfg.solver != AFS_SOLVER_TREE || hop < AFS_PLAN_HOP_MIN)
    return fail(c, AFS_ERR_UNSUPPORTED, "afs_noise_plan_hops: tree solver and hop >= AFS_PLAN_HOP_MIN only");
  if (!frames || !hops || !plans || rows <= 0 || F < 2 || s0 < 0 || s1 <= s0 || s1 > (int64_t)(F - 1) * hop)
    return fail(c, AFS_ERR_INVALID_ARGUMENT, "afs_noise_plan_hops: need frames, hops, plans, rows>0, num_frames>=2, "
                                             "0 <= s_begin < s_end <= (num_frames-1)*hop");
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  afs_status s;
  const afs_frame *dframes = frames;
  if (!is_device_ptr(frames)) {
    const size_t bytes = (size_t)rows * F * sizeof(afs_frame);
    if ((s = ensure(c, &c->stage_in, &c->stage_in_bytes, bytes)) != AFS_OK) return s;
    HIP_TRY(c, hipMemcpyAsync(c->stage_in, frames, bytes, hipMemcpyHostToDevice, c->stream));
    dframes = (const afs_frame *)c->stage_in;
  }
  const int64_t n = s1 - s0, slots = afs::plan_hop_slots(s0, s1, hop);
  const size_t pbytes = (size_t)rows * (size_t)n * afs::PLAN_RECORD_BYTES;
  const size_t hbytes = (size_t)rows * (size_t)slots * sizeof(afs::tree::PlanHop);
  uint64_t *dplans = plans;
  uint8_t *dhops = hops;
  const bool host_plans = !is_device_ptr(plans), host_hops = !is_device_ptr(hops);
  if (host_plans) {
    if ((s = ensure(c, &c->plan, &c->plan_bytes, pbytes)) != AFS_OK) return s;
    dplans = (uint64_t *)c->plan;
    HIP_TRY(c, hipMemcpyAsync(dplans, plans, pbytes, hipMemcpyHostToDevice, c->stream));
  }
  if (host_hops) {
    if ((s = ensure(c, &c->hops[0], &c->hops_bytes[0], hbytes)) != AFS_OK) return s;
    dhops = (uint8_t *)c->hops[0];
  }
  if ((s = ensure(c, &c->plan_work[0], &c->plan_work_bytes[0], (size_t)afs::plan_work_bytes(rows, slots))) != AFS_OK)
    return s;
  afs::PlanArgs pa{c->dev_tab, dframes, F, rows, hop, s0, s1, dplans, n,
                   c->cfg.options.glottis_model == AFS_GLOTTIS_TWO_MASS ? 1 : 0, c->dev_tab->consts.sec,
                   (afs::tree::PlanHop *)dhops, slots, (uint32_t *)c->plan_work[0]};
  HIP_TRY(c, afs::launch_plan_hops(pa, c->stream));
  if (host_plans) HIP_TRY(c, hipMemcpyAsync(plans, dplans, pbytes, hipMemcpyDeviceToHost, c->stream));
  if (host_hops) HIP_TRY(c, hipMemcpyAsync(hops, dhops, hbytes, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return AFS_OK;
}

afs_status afs_plan_hop_words(afs_ctx *c, const uint8_t *hops, const double *ratio, int32_t n, uint64_t *words) {
  if (!c) return AFS_ERR_INVALID_ARGUMENT;
  if (c->cfg.solver != AFS_SOLVER_TREE) return fail(c, AFS_ERR_UNSUPPORTED, "afs_plan_hop_words: tree solver only");
  if (!hops || !ratio || !words || n <= 0)
    return fail(c, AFS_ERR_INVALID_ARGUMENT, "afs_plan_hop_words: need hops, ratio, words, n>0");
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  const size_t hb = (size_t)n * sizeof(afs::tree::PlanHop), rb = (size_t)n * 8, wb = (size_t)n * AFS_PLAN_WORDS * 8;
  char *d = nullptr;
  HIP_TRY(c, hipMalloc((void **)&d, hb + rb + wb));
  hipError_t e = hipMemcpyAsync(d, hops, hb, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(d + hb, ratio, rb, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess)
    e = afs::launch_tree_hop_words((const afs::tree::PlanHop *)d, (const double *)(d + hb), n, (uint64_t *)(d + hb + rb),
                                   c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(words, d + hb + rb, wb, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(d);
  HIP_TRY(c, e);
  return AFS_OK;
}

afs_status afs_tube_interpolate(afs_ctx *c, const afs_frame *fl, const afs_frame *fr, const double *ratio, int32_t n,
                                double *area, double *length) {
  if (!c) return AFS_ERR_INVALID_ARGUMENT;
  if (c->cfg.solver != AFS_SOLVER_TREE) return fail(c, AFS_ERR_UNSUPPORTED, "afs_tube_interpolate: tree solver only");
  if (!fl || !fr || !ratio || !area || !length || n <= 0)
    return fail(c, AFS_ERR_INVALID_ARGUMENT, "afs_tube_interpolate: need left, right, ratio, area, length, n>0");
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  const size_t fb = (size_t)n * sizeof(afs_frame), rb = (size_t)n * 8, ob = (size_t)n * AFS_NUM_TUBE_SECTIONS * 8;
  char *d = nullptr;
  HIP_TRY(c, hipMalloc((void **)&d, 2 * fb + rb + 2 * ob));
  afs_frame *dl = (afs_frame *)d, *dr = (afs_frame *)(d + fb);
  double *dratio = (double *)(d + 2 * fb), *da = (double *)(d + 2 * fb + rb), *dlen = (double *)(d + 2 * fb + rb + ob);
  hipError_t e = hipMemcpyAsync(dl, fl, fb, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(dr, fr, fb, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(dratio, ratio, rb, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemsetAsync(da, 0, 2 * ob, c->stream);
  if (e == hipSuccess) e = afs::launch_tree_interp(c->dev_tab, dl, dr, dratio, n, da, dlen, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(area, da, ob, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(length, dlen, ob, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(d);
  HIP_TRY(c, e);
  return AFS_OK;
}

afs_status afs_session_create(afs_ctx *c, int32_t B, const uint32_t *seeds, afs_session **out) {
  if (!c || !out || B <= 0) return c ? fail(c, AFS_ERR_INVALID_ARGUMENT, "afs_session_create: bad args") : AFS_ERR_INVALID_ARGUMENT;
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  afs_session *s = new afs_session();
  s->ctx = c;
  s->B = B;
  s->bp = pad64(B);
  s->lanes = lanes_for(c, B);  // (fixed for the session: the per-lane state layout depends on it)
  auto bail = [&](hipError_t e) {
    afs_session_destroy(s);
    return fail(c, e == hipErrorOutOfMemory ? AFS_ERR_OUT_OF_MEMORY : AFS_ERR_HIP, "session alloc: %s", hipGetErrorString(e));
  };
  hipError_t e;
  if ((e = hipMalloc(&s->ws, ws_bytes_for(c, s->bp))) != hipSuccess) return bail(e);
  if ((e = hipMalloc((void **)&s->rng, (size_t)(32 * s->bp) * sizeof(int32_t))) != hipSuccess) return bail(e);
  if (tree(c) && (e = hipMalloc(&s->tree_lanes, lanes_bytes_for(c, s->bp, s->lanes))) != hipSuccess) return bail(e);
  if ((e = hipMalloc((void **)&s->pair, (size_t)B * 2 * sizeof(afs_frame))) != hipSuccess) return bail(e);
  if ((e = hipMalloc((void **)&s->seeds, (size_t)B * sizeof(uint32_t))) != hipSuccess) return bail(e);
  if ((e = hipHostMalloc((void **)&s->hframes, (size_t)B * sizeof(afs_frame), hipHostMallocDefault)) != hipSuccess)
    return bail(e);
  *out = s;
  afs_status st = afs_session_reset(s, seeds);
  if (st != AFS_OK) {
    afs_session_destroy(s);
    *out = nullptr;
  }
  return st;
}

afs_status afs_session_reset(afs_session *s, const uint32_t *seeds) {
  if (!s) return AFS_ERR_INVALID_ARGUMENT;
  afs_ctx *c = s->ctx;
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  if (seeds) {
    hipMemcpyKind k = is_device_ptr(seeds) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    HIP_TRY(c, hipMemcpyAsync(s->seeds, seeds, (size_t)s->B * 4, k, c->stream));
  }
  // (no seeds: the reset kernels seed voice u with u + 1)
  afs_status st = reset_state(c, s->ws, s->rng, s->tree_lanes, s->bp, s->B, seeds ? s->seeds : nullptr, s->lanes);
  if (st != AFS_OK) return st;
  s->latched = false;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return AFS_OK;
}

void afs_session_destroy(afs_session *s) {
  if (!s) return;
  if (s->ws) (void)hipFree(s->ws);
  if (s->rng) (void)hipFree(s->rng);
  if (s->tree_lanes) (void)hipFree(s->tree_lanes);
  if (s->pair) (void)hipFree(s->pair);
  if (s->seeds) (void)hipFree(s->seeds);
  if (s->hframes) (void)hipHostFree(s->hframes);
  if (s->hout) (void)hipHostFree(s->hout);
  delete s;
}

afs_status afs_session_synthesize(afs_session *s, const afs_frame *frames, int32_t n, double *out,
                                  uint8_t *nonfinite, int32_t *produced, afs_report *rep) {
  if (!s || !frames) return AFS_ERR_INVALID_ARGUMENT;
  afs_ctx *c = s->ctx;
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  const int B = s->B;
  // (the kinds of the caller's pointers are probed on every call: a freed buffer's address may come
  // back as memory of the other kind; one pointer query is ~1 us beside a ~6 ms call)
  const bool in_dev = is_device_ptr(frames);
  const afs_frame *src = frames;
  if (!in_dev) {  // host frames: through the session's pinned buffer
    std::memcpy(s->hframes, frames, (size_t)B * sizeof(afs_frame));
    src = s->hframes;
  }
  const hipMemcpyKind k = in_dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  // frames[u] -> pair[u][slot]
  const int slot = s->latched ? 1 : 0;
  HIP_TRY(c, hipMemcpy2DAsync(s->pair + slot, 2 * sizeof(afs_frame), src, sizeof(afs_frame),
                              sizeof(afs_frame), B, k, c->stream));
  if (!s->latched) {  // Synthesizer.cpp:522-532
    s->latched = true;
    if (produced) *produced = 0;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (rep) { std::memset(rep, 0, sizeof *rep); rep->kernel = c->cfg.solver; }
    return AFS_OK;
  }
  if (!out) return fail(c, AFS_ERR_INVALID_ARGUMENT, "afs_session_synthesize: out is NULL");
  if (n < 1) n = 1;  // Synthesizer.cpp:543-546
  double *dout = out;
  const bool host_out = !is_device_ptr(out);
  const size_t nout = (size_t)B * (size_t)n;
  afs_status st;
  if (host_out) {
    if ((st = ensure(c, &c->stage_out, &c->stage_out_bytes, nout * sizeof(double))) != AFS_OK) return st;
    dout = (double *)c->stage_out;
    if (nout > s->hout_cap) {
      if (s->hout) (void)hipHostFree(s->hout);
      s->hout = nullptr;
      s->hout_cap = 0;
      HIP_TRY(c, hipHostMalloc((void **)&s->hout, nout * sizeof(double), hipHostMallocDefault));
      s->hout_cap = nout;
    }
  }
  HIP_TRY(c, hipEventRecord(c->ev0, c->stream));
  if ((st = run_chunks(c, s->pair, 2, B, 1, n, dout, n, s->ws, s->rng, s->tree_lanes, s->bp, B, s->lanes, nullptr,
                       plain_order(c))) != AFS_OK)
    return st;
  HIP_TRY(c, hipEventRecord(c->ev1, c->stream));
  // prevTube = *newTube (Synthesizer.cpp:633-637)
  HIP_TRY(c, hipMemcpy2DAsync(s->pair, 2 * sizeof(afs_frame), s->pair + 1, 2 * sizeof(afs_frame),
                              sizeof(afs_frame), B, hipMemcpyDeviceToDevice, c->stream));
  bool nf_sync = false;
  if ((st = nonfinite_report(c, s->ws, s->bp, B, nonfinite, rep != nullptr, &nf_sync)) != AFS_OK) return st;
  if (host_out) HIP_TRY(c, hipMemcpyAsync(s->hout, dout, nout * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (host_out) std::memcpy(out, s->hout, nout * sizeof(double));
  if (produced) *produced = n;
  if (rep) {
    float ms = 0.f;
    HIP_TRY(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
    rep->device_ms = ms;
    rep->samples = (int64_t)B * n;
    rep->nonfinite_utterances = *c->hcount;
    rep->kernel = c->cfg.solver;
  }
  return AFS_OK;
}

afs_status afs_session_rng_draws(afs_session *s, int64_t *draws) {
  if (!s || !draws) return AFS_ERR_INVALID_ARGUMENT;
  afs_ctx *c = s->ctx;
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  return draws_of(c, s->ws, s->B, draws);
}

afs_status afs_af_to_frames(afs_ctx *c, const double *params, int64_t n, afs_frame *frames) {
  if (!c) return AFS_ERR_INVALID_ARGUMENT;
  if (!params || !frames || n <= 0) return fail(c, AFS_ERR_INVALID_ARGUMENT, "afs_af_to_frames: bad args");
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  const double *dp = params;
  void *tmp_p = nullptr, *tmp_f = nullptr;
  const bool host_p = !is_device_ptr(params), host_f = !is_device_ptr(frames);
  afs_frame *df = frames;
  if (host_p) {
    HIP_TRY(c, hipMalloc(&tmp_p, (size_t)n * 16 * sizeof(double)));
    HIP_TRY(c, hipMemcpyAsync(tmp_p, params, (size_t)n * 16 * sizeof(double), hipMemcpyHostToDevice, c->stream));
    dp = (const double *)tmp_p;
  }
  if (host_f) {
    HIP_TRY(c, hipMalloc(&tmp_f, (size_t)n * sizeof(afs_frame)));
    HIP_TRY(c, hipMemcpyAsync(tmp_f, frames, (size_t)n * sizeof(afs_frame), hipMemcpyHostToDevice, c->stream));
    df = (afs_frame *)tmp_f;
  }
  HIP_TRY(c, afs::launch_af_to_frames(dp, n, df, c->stream));
  if (host_f) HIP_TRY(c, hipMemcpyAsync(frames, df, (size_t)n * sizeof(afs_frame), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (tmp_p) (void)hipFree(tmp_p);
  if (tmp_f) (void)hipFree(tmp_f);
  return AFS_OK;
}

afs_status afs_to_int16(afs_ctx *c, const double *samples, int64_t n, int16_t *out) {
  if (!c) return AFS_ERR_INVALID_ARGUMENT;
  if (n == 0) return AFS_OK;  // empty views may carry null pointers
  if (!samples || !out || n < 0) return fail(c, AFS_ERR_INVALID_ARGUMENT, "afs_to_int16: bad args");
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  const bool host_in = !is_device_ptr(samples), host_out = !is_device_ptr(out);
  struct Staging {  // freed on every return path
    void *in = nullptr, *out = nullptr;
    ~Staging() {
      if (in) (void)hipFree(in);
      if (out) (void)hipFree(out);
    }
  } tmp;
  const double *din = samples;
  int16_t *dout = out;
  if (host_in) {
    HIP_TRY(c, hipMalloc(&tmp.in, (size_t)n * sizeof(double)));
    HIP_TRY(c, hipMemcpyAsync(tmp.in, samples, (size_t)n * sizeof(double), hipMemcpyHostToDevice, c->stream));
    din = (const double *)tmp.in;
  }
  if (host_out) {
    HIP_TRY(c, hipMalloc(&tmp.out, (size_t)n * sizeof(int16_t)));
    dout = (int16_t *)tmp.out;
  }
  HIP_TRY(c, afs::launch_to_int16(din, dout, n, c->stream));
  if (host_out) HIP_TRY(c, hipMemcpyAsync(out, dout, (size_t)n * sizeof(int16_t), hipMemcpyDeviceToHost, c->stream));
  if (host_in || host_out || !(c->cfg.flags & AFS_ASYNC)) HIP_TRY(c, hipStreamSynchronize(c->stream));
  return AFS_OK;
}

// ---- Synthesizer::playTargetSequence (Synthesizer.cpp:1299-1422) -------------------------

void afs_target_sequence_default(afs_target_sequence *ts) {
  if (!ts) return;
  static const double st[4] = {0.2, 0.05, 0.2, 0.1}, tr[3] = {0.05, 0.05, 0.05}, f0[4] = {100, 115, 105, 80};
  static const double g[6] = {120.0, 10000.0, 0.01, 0.01, 0.0, -40.0};
  std::memcpy(ts->stationary_s, st, sizeof st);
  std::memcpy(ts->transition_s, tr, sizeof tr);
  std::memcpy(ts->f0_hz, f0, sizeof f0);
  ts->lung_pressure_dpa = 8000.0;
  std::memcpy(ts->glottis, g, sizeof g);
}

static void target_bounds(const afs_target_sequence *ts, double *b) {  // :1318-1326, left to right
  const double *s = ts->stationary_s, *t = ts->transition_s;
  b[0] = s[0];
  b[1] = s[0] + t[0];
  b[2] = s[0] + t[0] + s[1];
  b[3] = s[0] + t[0] + s[1] + t[1];
  b[4] = s[0] + t[0] + s[1] + t[1] + s[2];
  b[5] = s[0] + t[0] + s[1] + t[1] + s[2] + t[2];
  b[6] = s[0] + t[0] + s[1] + t[1] + s[2] + t[2] + s[3];
}

int64_t afs_target_sequence_samples(const afs_target_sequence *ts, double fs) {
  if (!ts || !(fs > 0.0)) return -1;
  double b[7];
  target_bounds(ts, b);
  const double n = fs * b[6];
  if (!(n >= 0.0) || n >= 2147483647.0) return -1;
  return (int64_t)(int)n;  // int numSamples = SAMPLING_RATE * totalTime_s
}

afs_status afs_play_target_sequences(afs_ctx *c, const double *shapes, int32_t num_shapes, const int32_t *targets,
                                     const afs_target_sequence *ts, const uint32_t *seeds, int32_t B, double *out,
                                     uint8_t *nonfinite, afs_report *rep) {
  if (!c) return AFS_ERR_INVALID_ARGUMENT;
  if (!shapes || num_shapes <= 0 || !targets || !ts || B <= 0 || !out)
    return fail(c, AFS_ERR_INVALID_ARGUMENT, "afs_play_target_sequences: need shapes, targets, timing, batch>0, out");
  if (is_device_ptr(shapes) || is_device_ptr(targets))
    return fail(c, AFS_ERR_INVALID_ARGUMENT, "afs_play_target_sequences: shapes and targets are host arrays");
  const double fs = c->cfg.sampling_rate_hz;
  const int64_t T = afs_target_sequence_samples(ts, fs);
  if (T < 0) return fail(c, AFS_ERR_INVALID_ARGUMENT, "afs_play_target_sequences: bad timing");
  for (int64_t k = 0; k < (int64_t)B * 4; ++k)
    if (targets[k] < 0 || targets[k] >= num_shapes)
      return fail(c, AFS_ERR_INVALID_ARGUMENT, "afs_play_target_sequences: target %lld out of range", (long long)k);
  if (rep) std::memset(rep, 0, sizeof *rep);
  if (T == 0) {
    if (nonfinite) {
      if (is_device_ptr(nonfinite)) HIP_TRY(c, hipMemset(nonfinite, 0, (size_t)B));
      else std::memset(nonfinite, 0, (size_t)B);
    }
    return AFS_OK;
  }
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  // one tube trajectory per distinct sequence of four shapes
  std::map<std::array<int32_t, 4>, int32_t> uniq;
  std::vector<int32_t> row((size_t)B);
  std::vector<double> seq;
  for (int32_t b = 0; b < B; ++b) {
    const std::array<int32_t, 4> key{targets[4 * b], targets[4 * b + 1], targets[4 * b + 2], targets[4 * b + 3]};
    auto it = uniq.find(key);
    if (it == uniq.end()) {
      it = uniq.emplace(key, (int32_t)uniq.size()).first;
      for (int j = 0; j < 4; ++j) seq.insert(seq.end(), shapes + 16 * (int64_t)key[j], shapes + 16 * (int64_t)key[j] + 16);
    }
    row[(size_t)b] = it->second;
  }
  const int Q = (int)uniq.size();
  afs::TargetPlan plan{};
  target_bounds(ts, plan.b);
  plan.fs = fs;
  std::memcpy(plan.f0, ts->f0_hz, sizeof plan.f0);
  plan.P = ts->lung_pressure_dpa;
  std::memcpy(plan.glottis, ts->glottis, sizeof plan.glottis);
  {  // the last sample below 0.1 fs: its fade-in value is held until the fade-out
    int64_t j = (int64_t)std::ceil((double)0.1 * fs);
    while (j >= 0 && !((double)j < (double)0.1 * fs)) --j;
    while ((double)(j + 1) < (double)0.1 * fs) ++j;
    plan.hold_j = j;
  }
  afs_status s;
  const int width = lanes_for(c, B);
  // tree solver: the XCD-aware slot order of the utterances by trajectory (xcd_order)
  std::vector<int32_t> order;
  if (tree(c) && c->xcd_order) {
    const int upb = width == afs::TREE_VOICE_W ? 1 : afs::TREE_UPB;
    // blocks the GPU holds at once: the voice kernel one wave (block) per SIMD, the throughput
    // kernel one wave per SIMD in blocks of TREE_WPB waves (4 / TREE_WPB blocks per CU, its LDS)
    const int conc = width == afs::TREE_VOICE_W ? c->simds : c->simds / afs::TREE_WPB;
    order = xcd_order(row, B, upb, conc);
  }
  const size_t seq_bytes = seq.size() * sizeof(double);
  const size_t row_bytes = (size_t)B * sizeof(int32_t), ord_bytes = order.size() * sizeof(int32_t);
  if ((s = ensure(c, &c->tgt, &c->tgt_bytes, seq_bytes + row_bytes + ord_bytes)) != AFS_OK) return s;
  double *dseq = (double *)c->tgt;
  int32_t *drow = (int32_t *)((char *)c->tgt + seq_bytes);
  int32_t *dord = order.empty() ? nullptr : (int32_t *)((char *)c->tgt + seq_bytes + row_bytes);
  HIP_TRY(c, hipMemcpyAsync(dseq, seq.data(), seq_bytes, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipMemcpyAsync(drow, row.data(), row_bytes, hipMemcpyHostToDevice, c->stream));
  if (dord) HIP_TRY(c, hipMemcpyAsync(dord, order.data(), ord_bytes, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));  // the host vectors die with this call
  const uint32_t *dseeds = seeds;
  if (seeds && !is_device_ptr(seeds)) {
    if ((s = ensure(c, &c->stage_seeds, &c->stage_seeds_bytes, (size_t)B * 4)) != AFS_OK) return s;
    HIP_TRY(c, hipMemcpyAsync(c->stage_seeds, seeds, (size_t)B * 4, hipMemcpyHostToDevice, c->stream));
    dseeds = (const uint32_t *)c->stage_seeds;
  }
  double *dout = out;
  const bool host_out = !is_device_ptr(out);
  if (host_out) {
    if ((s = ensure(c, &c->stage_out, &c->stage_out_bytes, (size_t)B * T * sizeof(double))) != AFS_OK) return s;
    dout = (double *)c->stage_out;
  }
  const int64_t bp = pad64(B);
  if ((s = ensure(c, &c->ws, &c->ws_bytes, ws_bytes_for(c, bp))) != AFS_OK) return s;
  if ((s = ensure(c, (void **)&c->rng, &c->rng_bytes, (size_t)(32 * bp) * sizeof(int32_t))) != AFS_OK) return s;
  if (tree(c) && (s = ensure(c, &c->tree_lanes, &c->tree_lanes_bytes, lanes_bytes_for(c, bp, width))) != AFS_OK)
    return s;
  if ((s = reset_state(c, c->ws, c->rng, c->tree_lanes, bp, B, dseeds, width)) != AFS_OK) return s;
  // time chunks of Tc samples: Tc + 1 frames per sequence (the first repeats the previous
  // chunk's last), at most 1 GiB of frames
  const int64_t budget = (int64_t)1 << 30;
  const int64_t Tc = std::max<int64_t>(1, std::min<int64_t>({T, 65536, budget / ((int64_t)Q * (int64_t)sizeof(afs_frame)) - 1}));
  if ((s = ensure(c, &c->stage_in, &c->stage_in_bytes, (size_t)Q * (size_t)(Tc + 1) * sizeof(afs_frame))) != AFS_OK)
    return s;
  afs_frame *dframes = (afs_frame *)c->stage_in;
  HIP_TRY(c, hipEventRecord(c->ev0, c->stream));
  for (int64_t k0 = 0; k0 < T; k0 += Tc) {
    const int nk = (int)std::min<int64_t>(Tc, T - k0);
    HIP_TRY(c, afs::launch_target_frames(dseq, Q, plan, k0, nk + 1, Tc + 1, dframes, c->stream));
    SlotOrder so = plain_order(c);
    so.order = dord;
    if ((s = run_chunks(c, dframes, Tc + 1, Q, nk, 1, dout + k0, T, c->ws, c->rng, c->tree_lanes, bp, B, width,
                        drow, so)) != AFS_OK)
      return s;
  }
  HIP_TRY(c, hipEventRecord(c->ev1, c->stream));
  c->last_B = B;
  bool nf_sync = false;
  if ((s = nonfinite_report(c, c->ws, bp, B, nonfinite, rep != nullptr, &nf_sync)) != AFS_OK) return s;
  if (host_out) HIP_TRY(c, hipMemcpyAsync(out, dout, (size_t)B * T * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  const bool sync = !(c->cfg.flags & AFS_ASYNC) || host_out || rep || nf_sync;
  if (sync) HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (rep) {
    float ms = 0.f;
    HIP_TRY(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
    rep->device_ms = ms;
    rep->samples = (int64_t)B * T;
    rep->nonfinite_utterances = *c->hcount;
    rep->kernel = c->cfg.solver;
  }
  return AFS_OK;
}

}  // extern "C"
