// afs_audio.h -- output format stage (audio_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace afs {

hipError_t launch_to_int16(const double *in, int16_t *out, int64_t n, hipStream_t st);
// load the code object on the current device (afs_create; see afs_tree.h)
hipError_t preload_audio_kernels();

}  // namespace afs
