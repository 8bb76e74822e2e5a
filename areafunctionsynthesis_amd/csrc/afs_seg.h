// afs_seg.h -- host-side interface of the segment-aligned kernel (tds_seg.hip, seg_core.h).
#pragma once

#include <hip/hip_runtime.h>

#include "afs_tree.h"
#include "seg_model.h"

namespace afs {

// The launch arguments of the tree kernel plus the seg tables (device copy).
struct SegArgs {
  TreeArgs t;
  const seg::SegTables *seg;
};

#ifndef AFS_SEG_WPB
#define AFS_SEG_WPB 4
#endif
int64_t seg_lane_bytes();
int64_t seg_lds_doubles();
hipError_t launch_seg_reset(void *lane_state, double *lds_state, int B, const uint32_t *seeds, hipStream_t st);
hipError_t launch_seg_synth(const SegArgs &a, hipStream_t st);
hipError_t launch_seg_nonfinite(const double *lds_state, int B, int32_t *count, uint8_t *flags, hipStream_t st);
hipError_t launch_seg_draws(const double *lds_state, int B, int64_t *draws, hipStream_t st);

}  // namespace afs
