// afs_tree.h -- host-side interface of the cooperative tree kernel (tds_tree.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "afs_model.h"
#include "tree_plan.h"

namespace afs {

// Sample s (0-based) of a call plays frame transition k = 1 + s / hop (frames k-1, k of the
// utterance's row) at ratio (s % hop) / hop; a launch covers samples [s_begin, s_end).
struct TreeArgs {
  const Tables *tab;
  const afs_frame *frames;  // frames[row(u) * frame_stride + k]
  int64_t frame_stride;
  const int32_t *frame_row; // row(u) = frame_row[u], or u when null (shared trajectories)
  int hop;
  int64_t s_begin, s_end;
  double *out;              // out[u * out_stride + s - s_begin]
  int64_t out_stride;
  const uint64_t *plan;     // plan[(row(u) * plan_stride + s - s_begin) * 16 + w] (tree_plan.h); hop
                            // mode: the compact dense records of the mixed hops (PlanArgs::compact)
  int64_t plan_stride;
  void *lane_state;         // per-lane register state, B * lanes entries (Lane<lanes>)
  double *lds_state;        // per-utterance LDS block, B * tree_lds_doubles()
  int B;
  Uni uni;                  // copy of tab->uni: scalar kernel arguments
  // hop records (tree_plan.h PlanHop; null: every sample reads its dense record):
  // hops[row(u) * hop_stride + s / hop - s_begin / hop]; the dense records are written for the
  // samples of mixed hops only
  const tree::PlanHop *hops = nullptr;
  int64_t hop_stride = 0;
  // section 25's pressure per sample (p25[u * p25_stride + s - s_begin]), K6's glottal-tone input
  double *p25 = nullptr;
  int64_t p25_stride = 0;
  // utterance of slot block * (utterances per block) + g, or the identity when null (entries >= B:
  // padding slots); shared trajectories (frame_row) order the utterances by row so that the blocks
  // one XCD runs at a time play few rows (afs_capi.cpp xcd_order)
  const int32_t *order = nullptr;
  // hop mode: run each wave's launch in the lightest noise-phase variant its hop records allow
  // (tree_kernel.h noise_variant; 0: always the full phases -- AFS_NOISE_VARIANTS=0, A/B and tests)
  int noise_variants = 1;
  // blocks of the launch (0: enough for B utterances); with `order`, blocks whose slots are all
  // padding exit at once (the XCD-dealt slot order of afs_capi.cpp shape_order)
  int grid_blocks = 0;
  // the variant rule decided on the device (afs_capi.cpp shape_order: the call's slot order sorted
  // on the device): when set, *variants_dev replaces noise_variants
  const int32_t *variants_dev = nullptr;
  // hop mode with compact slots that may not hold every mixed hop (afs_capi.cpp run_chunks): the
  // launch does nothing when K5 claimed more than skip_cap slots (*skip_claims > skip_cap); the host
  // then runs the call through the chunked path instead
  const uint32_t *skip_claims = nullptr;
  int64_t skip_cap = 0;
  // wave pairs: when the STAT waves run at a higher issue priority than their SIMDs' DYN waves
  // (s_setprio; tree_core.h pair_prio): 0 never, 1 during the solver, 2 during the first phase group and
  // the solver, 3 the whole launch (afs_capi.cpp picks by the launch's rounds of workgroups per CU
  // slot; profiles/r06_pair_ab.txt r06zh-r06zm)
  int stat_prio = 0;
};
// K5: the noise-source plans of samples [s_begin, s_end) of `rows` frame rows.
struct PlanArgs {
  const Tables *tab;
  const afs_frame *frames;
  int64_t frame_stride;
  int rows, hop;
  int64_t s_begin, s_end;
  uint64_t *plan;           // as TreeArgs::plan
  int64_t plan_stride;
  int two_mass;
  const SecRec *uo;         // the synthesis kernel's LDS offsets of the section outputs' noise-
                            // smoothed flows (tab->consts.sec)
  tree::PlanHop *hops = nullptr;  // hop mode (launch_plan_hops): as TreeArgs::hops
  int64_t hop_stride = 0;
  uint32_t *work = nullptr;  // hop mode: work[0] the hops listed (decided sample by sample), work[1]
                             // the compact slots claimed, then rows * hop slots list entries
  // hop mode: the dense records of a mixed hop go to the next free slot e of a compact array
  // (plan[(e * hop + i) * 16 + w] for the hop's sample i; PlanHop::dense = e; e < dense_cap, else
  // nothing is written: the K1 / K6 launches guarded by work[1] do nothing and the host, which reads
  // work[1] back, falls back to shorter launches)
  // instead of sample-indexed rows (the diagnostics' layout)
  bool compact = false;
  int64_t dense_cap = 0;
};
constexpr int64_t PLAN_RECORD_BYTES = 128;
// Hop slots a launch of samples [s0, s1) spans.
inline int64_t plan_hop_slots(int64_t s0, int64_t s1, int hop) { return (s1 - 1) / hop - s0 / hop + 1; }
// Bytes of the hop-mode work list of a launch.
inline int64_t plan_work_bytes(int64_t rows, int64_t slots) { return (rows * slots + 2) * 4; }

#ifndef AFS_TREE_W
#define AFS_TREE_W 16
#endif
#ifndef AFS_PAIR
// 1: the throughput kernel as wave pairs (tree_kernel.h tree_pair_body): two waves per SIMD, the
// phases of each four utterances split between a DYN and a STAT wave -- +8.7 % at 8192 static
// vowels, the audio bitwise the same (profiles/r06_pair_ab.txt); 0: one wave per SIMD running every
// phase (tree_synth_body; A/B builds)
#define AFS_PAIR 1
#endif
#ifndef AFS_TONE_K6
// 1: K1 stores section 25's pressure per sample and K6 runs the glottal-tone filter over it
// (+0.5 % end to end in round 3, profiles/r03ai_ab.txt); 0: K1 runs the filter itself, per sample
// (A/B builds); 2: K1 runs it over each 16-sample output window when the window is stored, the tone
// added to the stored flows (tree_kernel.h tone_window; A/B builds)
#define AFS_TONE_K6 1
#endif
#ifndef AFS_TREE_WPB
// waves per block of the throughput kernel: 2 (8 utterances, 78 KB of LDS: two blocks per CU).  With
// the slot order by shape, finer blocks balance the compute units' two rounds better: +0.6 % static
// vowels against 4 (profiles/r04ab_wpb_ab.txt; without the order it measured neutral, r04p)
#define AFS_TREE_WPB 2
#endif
#ifndef AFS_TREE_MIN_WAVES
#define AFS_TREE_MIN_WAVES 1  // waves per SIMD the register allocation must allow
#endif
constexpr int TREE_W = AFS_TREE_W;      // lanes per utterance of the throughput kernel (16)
constexpr int TREE_WPB = AFS_TREE_WPB;  // its waves per block
constexpr int TREE_VOICE_W = 64;        // lanes per utterance of the voice kernel (one utterance per wave)
// Batches up to this many utterances run the voice kernel as wave pairs (AFS_PAIR builds: two waves
// per utterance on two SIMDs, 256 VGPRs each with the lean solver, so that a SIMD can hold two):
// one voice's 1102-sample call 5.0 instead of 6.4 ms, config 2 (1024 utterances) +4.4 %, the audio
// bitwise the one-wave kernel's (profiles/r06_pair_ab.txt r06z / r06za).  Larger batches that still
// take 64 lanes (AFS_LANES_64) run one wave per utterance.
#ifndef AFS_PAIR64_MAX
#define AFS_PAIR64_MAX 1024
#endif
#ifndef AFS_PAIR64_WAVES
#define AFS_PAIR64_WAVES 2  // waves per SIMD the voice pairs' registers must allow (1: the full solver, 282 VGPRs)
#endif
constexpr int TREE_PAIR64_MAX = AFS_PAIR64_MAX;
constexpr int TREE_UPB = (64 / TREE_W) * TREE_WPB;  // utterances per block of the throughput kernel
// Lanes per utterance: TREE_W or TREE_VOICE_W (the per-lane state layout, Lane<lanes>, differs).
int64_t tree_lane_bytes(int lanes);
int64_t tree_lds_doubles();
hipError_t launch_tree_reset(void *lane_state, double *lds_state, int B, const uint32_t *seeds, int lanes,
                             hipStream_t st);
hipError_t launch_tree_synth(const TreeArgs &a, int lanes, hipStream_t st);
// K6, after each tree_synth launch of samples [s_begin, s_end): the glottal-tone filter over the
// section-25 pressures (p25, skin != 0) and the output stage over the flows the launch stored
// (out[u * out_stride + s - s_begin], replaced by the audio).
// (skip_claims: as TreeArgs::skip_claims -- the launch does nothing when *skip_claims > skip_cap)
hipError_t launch_tree_output(const Tables *tab, double *lds_state, double *out, int64_t out_stride, int64_t n, int B,
                              const double *p25, int64_t p25_stride, int skin, hipStream_t st,
                              const uint32_t *skip_claims = nullptr, int64_t skip_cap = 0);
// Load the tree kernels' and K5's code objects on the current device (afs_create: no code-object
// load inside the first synthesis call).
hipError_t preload_tree_kernels();
hipError_t preload_plan_kernels();
hipError_t launch_tree_nonfinite(const double *lds_state, int B, int32_t *count, uint8_t *flags, hipStream_t st);
hipError_t launch_tree_draws(const double *lds_state, int B, int64_t *draws, hipStream_t st);
hipError_t launch_plan(const PlanArgs &a, hipStream_t st);
// K5 in hop mode: the hop records of the launch's hops, the dense records of its mixed hops
hipError_t launch_plan_hops(const PlanArgs &a, hipStream_t st);
// ... in its two stages: the interval decisions (records of the decided hops, the work list of the
// others; a.work[0] = its length) and the per-sample decisions of the listed hops
hipError_t launch_plan_hops_iv(const PlanArgs &a, hipStream_t st);
hipError_t launch_plan_hops_wave(const PlanArgs &a, hipStream_t st);
// diagnostics: the tree kernel's per-sample plan words from hop records (afs_plan_hop_words)
hipError_t launch_tree_hop_words(const tree::PlanHop *h, const double *ratio, int n, uint64_t *out, hipStream_t st);
// diagnostics: the tree kernel's tube interpolation (afs_tube_interpolate)
hipError_t launch_tree_interp(const Tables *tab, const afs_frame *fl, const afs_frame *fr, const double *ratio, int n,
                              double *area, double *len, hipStream_t st);

}  // namespace afs
