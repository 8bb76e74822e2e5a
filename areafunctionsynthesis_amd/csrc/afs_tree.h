// afs_tree.h -- host-side interface of the cooperative tree kernel (tds_tree.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "afs_model.h"

namespace afs {

struct TreeArgs {
  const Tables *tab;
  const afs_frame *frames;  // frames[row(u) * frame_stride + k]
  int64_t frame_stride;
  const int32_t *frame_row; // row(u) = frame_row[u], or u when null (shared trajectories)
  int k_begin, k_end, hop;
  double *out;              // out[u * out_stride + t]
  int64_t out_stride;
  void *lane_state;         // per-lane register state, B * TREE_W entries
  double *lds_state;        // per-utterance LDS block, B * tree_lds_doubles()
  int B;
  Uni uni;                  // copy of tab->uni: scalar kernel arguments
};

#ifndef AFS_TREE_W
#define AFS_TREE_W 16
#endif
#ifndef AFS_TREE_WPB
#define AFS_TREE_WPB 4
#endif
#ifndef AFS_TREE_MIN_WAVES
#define AFS_TREE_MIN_WAVES 1  // waves per SIMD the register allocation must allow
#endif
constexpr int TREE_W = AFS_TREE_W;      // lanes per utterance (16 or 32)
constexpr int TREE_WPB = AFS_TREE_WPB;  // waves per block
int64_t tree_lane_bytes();
int64_t tree_lds_doubles();
hipError_t launch_tree_reset(void *lane_state, double *lds_state, int B, const uint32_t *seeds, hipStream_t st);
hipError_t launch_tree_synth(const TreeArgs &a, hipStream_t st);
hipError_t launch_tree_nonfinite(const double *lds_state, int B, int32_t *count, hipStream_t st);

}  // namespace afs
