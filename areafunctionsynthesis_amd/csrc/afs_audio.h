// afs_audio.h -- output format stage (audio_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace afs {

hipError_t launch_to_int16(const double *in, int16_t *out, int64_t n, hipStream_t st);

}  // namespace afs
