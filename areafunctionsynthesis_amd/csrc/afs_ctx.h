// afs_ctx.h -- the library's internal context and session objects (afs_capi.cpp,
// afs_comm.cpp) and the host helpers they share.  Not part of the C ABI.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "afs_model.h"

struct afs_ctx {
  afs_config cfg{};
  int simds = 1024;  // SIMDs of the device (the voice kernel's batch limit, afs_capi.cpp lanes_for)
  hipStream_t stream = nullptr;
  afs::Tables host_tab{};
  afs::Tables *dev_tab = nullptr;
  std::string err;
  // reusable device buffers for whole-trajectory calls
  void *ws = nullptr;
  size_t ws_bytes = 0;
  int32_t *rng = nullptr;
  size_t rng_bytes = 0;
  void *tree_lanes = nullptr;  // tree solver: per-lane register state
  size_t tree_lanes_bytes = 0;
  void *stage_in = nullptr;
  size_t stage_in_bytes = 0;
  void *stage_out = nullptr;
  size_t stage_out_bytes = 0;
  void *stage_seeds = nullptr;
  size_t stage_seeds_bytes = 0;
  void *tgt = nullptr;  // target sequences: shape rows [Q][4][16] then frame_row [B]
  size_t tgt_bytes = 0;
  void *plan = nullptr;   // tree solver: noise-source plans of one launch (tree_plan.h)
  size_t plan_bytes = 0;
  void *plan2 = nullptr;  // the second plan buffer: K5 fills one while K1 reads the other
  size_t plan2_bytes = 0;
  void *hops[2] = {nullptr, nullptr};  // tree solver, hops >= PLAN_HOP_MIN: hop records (tree_plan.h PlanHop)
  size_t hops_bytes[2] = {0, 0};
  void *p25 = nullptr;  // tree solver: section 25's pressure per sample of a launch (K6's tone input)
  size_t p25_bytes = 0;
  void *plan_work[2] = {nullptr, nullptr};  // hop mode: K5's work lists (the hops decided sample by sample)
  size_t plan_work_bytes[2] = {0, 0};
  bool plan_dense = false;             // AFS_PLAN_DENSE=1: dense records at every hop (A/B, tests)
  bool xcd_order = true;               // AFS_XCD_ORDER=0: shared trajectories in utterance order (A/B)
  int64_t launch_cap = 65536;          // samples per K1 launch at most (AFS_LAUNCH_SAMPLES lowers it)
  bool shape_order = true;             // AFS_SHAPE_ORDER=0: afs_synthesize's utterances in call order
  // AFS_NOISE_VARIANTS: 1 (default) K1's noise-phase variants for the calls whose slot order finds
  // at least half of the utterances in a light class (shape_order), 2 for every call, 0 never
  int noise_variants = 1;
  int class_order = 2;                 // AFS_CLASS_ORDER: the slot order's noise-class key (af_kernels.hip; A/B)
  int stat_prio = -1;                  // AFS_STAT_PRIO: the pairs' STAT priority mode (afs_tree.h), -1 by the launch's rounds
  void *keys = nullptr;                // shape keys, sorted keys, utterance indices, the variant flag (device)
  size_t keys_bytes = 0;
  void *sort_tmp = nullptr;            // the device radix sort's scratch
  size_t sort_tmp_bytes = 0;
  void *order_buf = nullptr;           // the slot order built from them (device)
  size_t order_bytes = 0;
  std::vector<uint64_t> hkeys;
  std::vector<int32_t> horder;
  hipStream_t plan_stream = nullptr;  // K5 of the next launch, beside K1 of this one (overlap)
  bool overlap = false;                // AFS_PLAN_OVERLAP=1 (afs_capi.cpp run_chunks)
  hipEvent_t ev_go = nullptr, ev_plan[2] = {nullptr, nullptr}, ev_free[2] = {nullptr, nullptr};
  hipEvent_t ev_k5 = nullptr;  // after K5 and the read-back of its claimed slots (run_chunks' guarded fast path)
  int64_t plan_budget = 0;  // bytes of plans one launch may use (afs_capi.cpp)
  void *stage_nf = nullptr;  // per-utterance non-finite flags staged for a host array
  size_t stage_nf_bytes = 0;
  // afs_multi_synthesize: this device's shard of float audio, its int16 audio, its flags, and
  // (device 0) the gathered int16 audio of the whole batch
  void *m_out = nullptr, *m_pcm = nullptr, *m_nf = nullptr, *m_root = nullptr;
  size_t m_out_bytes = 0, m_pcm_bytes = 0, m_nf_bytes = 0, m_root_bytes = 0;
  int32_t last_B = 0;        // batch of the last whole-trajectory call (afs_rng_draws)
  int32_t *dcount = nullptr;
  int32_t *hcount = nullptr;  // pinned host copy of dcount
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // AFS_PROFILE: an event pair around every kernel launch of the synthesis calls
  struct Timed { hipEvent_t a, b; int kind; };  // kind 0: synthesis kernel (K1), 1: noise-source plan (K5),
                                                // 2: output stage (K6)
  std::vector<hipEvent_t> pev;  // pool
  size_t pev_used = 0;
  std::vector<Timed> timed;
  bool timed_overflow = false;
};

struct afs_session {
  afs_ctx *ctx = nullptr;
  int B = 0;
  int64_t bp = 0;
  void *ws = nullptr;          // lane solver: SoA workspace; tree solver: per-utterance LDS blocks
  int32_t *rng = nullptr;      // lane solver: generator state; tree solver: unused
  void *tree_lanes = nullptr;  // tree solver: per-lane register state
  int lanes = 16;              // tree solver: lanes per utterance (fixed at creation)
  afs_frame *pair = nullptr;   // [B][2]: previous frame, new frame
  uint32_t *seeds = nullptr;   // device copy
  bool latched = false;
  // pinned staging of host frames and host output (a real-time caller's per-call copies go
  // through these instead of pageable memory)
  afs_frame *hframes = nullptr;
  double *hout = nullptr;
  size_t hout_cap = 0;  // doubles
};

namespace afs {

afs_status fail(afs_ctx *c, afs_status s, const char *fmt, ...);
bool is_device_ptr(const void *p);
afs_status ensure(afs_ctx *c, void **buf, size_t *cap, size_t bytes);
// afs_synthesize queued without a host wait (unless host buffers need one), with the tree solver's
// lanes per utterance fixed by the caller (lanes > 0; afs_multi_synthesize: the global batch's, so
// that a shard's audio does not depend on the GPU count) or chosen for B (lanes = 0)
afs_status synthesize_async(afs_ctx *c, const afs_frame *frames, const uint32_t *seeds, int32_t B, int32_t F,
                            int32_t hop, double *out, uint8_t *nonfinite, int lanes = 0);
// the lanes per utterance of the tree kernel for a batch of B (AFS_LANES_* or the library's choice)
int lanes_for(const afs_ctx *c, int64_t B);

}  // namespace afs

#define HIP_TRY(ctx, call)                                                                   \
  do {                                                                                       \
    hipError_t e_ = (call);                                                                  \
    if (e_ != hipSuccess)                                                                    \
      return afs::fail((ctx), e_ == hipErrorOutOfMemory ? AFS_ERR_OUT_OF_MEMORY : AFS_ERR_HIP, \
                       "%s failed: %s", #call, hipGetErrorString(e_));                       \
  } while (0)
