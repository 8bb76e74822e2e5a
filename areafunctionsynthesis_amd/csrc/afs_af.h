// afs_af.h -- host interface of the area-function kernels (af_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "afs_model.h"

namespace afs {

// OneDimAreaFunction parameters[n][16] -> the pharynx/mouth part of frames[n] (K2).
hipError_t launch_af_to_frames(const double *params, int64_t n, afs_frame *frames, hipStream_t st);

// Synthesizer::playTargetSequence's trajectory (Synthesizer.cpp:1299-1422), everything that
// does not depend on the target shapes, evaluated once on the host.
struct TargetPlan {
  double b[7];            // boundary_s (:1318-1326), summed left to right
  double fs;              // SAMPLING_RATE
  double f0[4];           // f0_Hz (:1311)
  double P;               // steadyStateLungPressure
  double glottis[6];      // init() latch glottis; [2..5] for every sample
  int64_t hold_j;         // the last sample index below 0.1 fs (its fade-in value is held)
};

// frames[q * fstride + k] = global frame k0 + k (k < n) of target sequence q, for Q sequences
// of 4 shapes each (seq[q][4][16]).  Frame 0 is init()'s schwa latch, frame g >= 1 is the tube
// and glottis controls of sample g - 1 (K4).
hipError_t launch_target_frames(const double *seq, int Q, const TargetPlan &plan, int64_t k0, int n,
                                int64_t fstride, afs_frame *frames, hipStream_t st);

// keys[u] = the shape key of utterance u's first frame frames[u * fstride] (how narrow its tube is
// and where), for the slot order of the tree kernel (afs_capi.cpp shape_order).
// (noise_class: 1 the noise class as the key's first field, 2 after the narrowness bucket, 0 not
// in the key; af_kernels.hip)
hipError_t launch_utterance_keys(const afs_frame *frames, int64_t fstride, int B, uint64_t *keys, int noise_class,
                                 hipStream_t st);

// The slot order on the device from keys[B] (launch_utterance_keys; overwritten): the variant rule
// (mode 0 never, 1 the rule, 2 always; the class field at bit `shift`, -1: none) into *variants, the
// utterances sorted stably by their (masked) keys into order[0 .. B), order[B .. slots) = B.
// keys_sorted[B], idx[B]: scratch.  temp == nullptr: only *temp_bytes is set (the sort's scratch).
hipError_t launch_slot_order(uint64_t *keys, uint64_t *keys_sorted, int32_t *idx, int B, int shift, int mode,
                             bool many_waves, int32_t *variants, int32_t *order, int slots, void *temp,
                             size_t *temp_bytes, hipStream_t st);

}  // namespace afs
