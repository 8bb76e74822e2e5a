// audio_kernels.hip -- the reference's output format stage.
//
// Synthesizer::synthesizeSegment (Synthesizer.cpp:955-973) stores every sample of
// synthesizeSignalTds in the int16 audio ring (Signal16 = TemplateSignal<signed short>,
// Signal.h:19, setValue :251) as short(x * SHRT_MAX), i.e. truncated towards zero, then
// clips x > 1 to SHRT_MAX and x < -1 to SHRT_MIN.  The double -> short conversion of a NaN
// is undefined in C++; on the reference's x86 build it yields 0, which is what we write.
// HBM-bound: 8 B in, 2 B out per sample; each thread converts 8 consecutive samples
// (one 16-byte store), so a wave moves 4 KB in and 1 KB out with coalesced accesses.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "afs_audio.h"

namespace afs {

__host__ __device__ inline int16_t sample_to_int16(double x) {
  if (x > 1.0) return 32767;
  if (x < -1.0) return -32768;
  if (!(x == x)) return 0;
  return (int16_t)(int)(x * 32767.0);  // |x| <= 1: fits; truncation towards zero
}

namespace {

__global__ void to_int16_kernel(const double *__restrict__ in, int16_t *__restrict__ out, int64_t n) {
  const int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i0 + 8 <= n) {
    int16_t v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = sample_to_int16(in[i0 + k]);
    if (((uintptr_t)(out + i0) & 15) == 0) {
      *(uint4 *)(out + i0) = *(const uint4 *)v;
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) out[i0 + k] = v[k];
    }
  } else {
    for (int64_t i = i0; i < n; ++i) out[i] = sample_to_int16(in[i]);
  }
}

}  // namespace

hipError_t launch_to_int16(const double *in, int16_t *out, int64_t n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t threads = (n + 7) / 8;
  const int64_t blocks = (threads + 255) / 256;
  hipLaunchKernelGGL(to_int16_kernel, dim3((unsigned)blocks), dim3(256), 0, st, in, out, n);
  return hipGetLastError();
}

// (see preload_tree_kernels, tds_tree.hip)
hipError_t preload_audio_kernels() {
  hipFuncAttributes at;
  return hipFuncGetAttributes(&at, reinterpret_cast<const void *>(to_int16_kernel));
}

}  // namespace afs
