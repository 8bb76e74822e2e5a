// af_kernels.hip -- the area-function model on the device (BASELINE row f1, kernel K2).
//
// OneDimAreaFunction::calculateArea (OneDimAreaFunction.cpp:23-58) and
// calculateOneDimTubeFunction (:75-138): 16 parameters -> 40 tube sections.  One lane
// per frame; the sequential sub-step walk x += step of the reference is kept as is,
// because the articulator classification depends on the exact accumulated x.
#include <cfloat>

#include <hip/hip_runtime.h>

#include "afs_lane.h"
#include "afs_model.h"

namespace afs {

namespace {

enum { P_LLAR, P_ALAR, P_POWLAR, P_XP, P_AP, P_POWP, P_XC, P_AC, P_POWC, P_XA, P_AA, P_POWA,
       P_XIN, P_AIN, P_LVT, P_ALIP };

__device__ double segment(double a1, double a0, double x1, double x0, double e, double x) {
  return (a1 + a0) / 2 + (a1 - a0) / 2 * cos(PI * pow((x1 - x) / (x1 - x0), e));
}

__device__ double af_area(const double *p, double x) {
  double a;
  if (x <= p[P_LLAR]) a = p[P_ALAR];
  else if (x <= p[P_XP]) a = segment(p[P_AP], p[P_ALAR], p[P_XP], p[P_LLAR], p[P_POWLAR], x);
  else if (x <= p[P_XC]) a = segment(p[P_AC], p[P_AP], p[P_XC], p[P_XP], p[P_POWP], x);
  else if (x <= p[P_XA]) a = segment(p[P_AA], p[P_AC], p[P_XA], p[P_XC], p[P_POWC], x);
  else if (x <= p[P_XIN]) a = segment(p[P_AIN], p[P_AA], p[P_XIN], p[P_XA], p[P_POWA], x);
  else a = p[P_ALIP];
  return a < 0.0 ? 0.0 : a;
}

__global__ void af_to_frames_kernel(const double *params, int64_t n, afs_frame *frames) {
  int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n) return;
  double p[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) p[i] = params[f * 16 + i];
  afs_frame *fr = frames + f;
  const double w = p[P_LVT] / 40;
  const double step = w * 0.01;
  double x = 0.0;
  for (int i = 0; i < NPM; ++i) {
    double mn = DBL_MAX;
    while (x < (i + 1) * w) {
      double a = af_area(p, x);
      if (a < mn) mn = a;
      x += step;
    }
    fr->length_cm[i] = w;
    fr->area_cm2[i] = mn;
    fr->laterality[i] = 0.0;
    uint8_t art;
    if (x <= p[P_XP]) art = OTHER;
    else if (x <= p[P_XIN] && x + w < p[P_XIN]) art = TONGUE;
    else if (x <= p[P_XIN]) art = LOWER_INCISORS;
    else art = LOWER_LIP;
    fr->articulator[i] = art;
  }
  fr->teeth_position_cm = p[P_XIN];
}

}  // namespace

hipError_t launch_af_to_frames(const double *params, int64_t n, afs_frame *frames, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(af_to_frames_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, params, n, frames);
  return hipGetLastError();
}

}  // namespace afs
