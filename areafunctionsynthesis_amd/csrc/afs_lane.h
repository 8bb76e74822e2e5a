// afs_lane.h -- host-side interface of the lane kernels (tds_lane.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "afs_model.h"

namespace afs {

struct LaneArgs {
  const Tables *tab;         // device copy of the tables
  const afs_frame *frames;   // frames[row(u) * frame_stride + k]
  int64_t frame_stride;
  const int32_t *frame_row;  // row(u) = frame_row[u], or u when null (shared trajectories)
  int k_begin, k_end;        // frame transitions (k-1 -> k) processed by this launch
  int hop;                   // samples per transition
  double *out;               // out[u * out_stride + t], t = 0 .. (k_end-k_begin)*hop-1
  int64_t out_stride;
  double *ws;                // SoA workspace, lane_ws_rows() rows of bp doubles
  int32_t *rng;              // 32 rows of bp ints (glibc TYPE_3 state + index)
  int64_t bp;                // padded batch (row pitch)
  int B;
  int sor;                   // 1: SOR (TdsModel::SOR_GAUSS_SEIDEL) instead of the Cholesky
};

int64_t lane_ws_rows(const Tables &t);
int64_t lane_persist_rows();
hipError_t launch_lane_reset(double *ws, int32_t *rng, int64_t bp, int B, const uint32_t *seeds, hipStream_t st);
hipError_t launch_lane_synth(const LaneArgs &a, hipStream_t st);
hipError_t launch_lane_nonfinite(const double *ws, int64_t bp, int B, int32_t *count, uint8_t *flags, hipStream_t st);

}  // namespace afs
