// af_kernels.hip -- the area-function model on the device.
//
// OneDimAreaFunction::calculateArea (OneDimAreaFunction.cpp:23-58) and
// calculateOneDimTubeFunction (:75-138): 16 parameters -> 40 tube sections.  One lane
// per frame; the sequential sub-step walk x += step of the reference is kept as is,
// because the articulator classification depends on the exact accumulated x.
#include <cfloat>

#include <hip/hip_runtime.h>
#include <hipcub/device/device_radix_sort.hpp>

#include "afs_af.h"
#include "afs_model.h"
#include "tree_plan.h"

#ifndef AFS_NZ_SET
#define AFS_NZ_SET 3  // (tree_core.h)
#endif

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

// calculateOneDimTubeFunction (:75-138) for one parameter vector.
__device__ void af_frame(const double *p, afs_frame *fr) {
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

__global__ void af_to_frames_kernel(const double *params, int64_t n, afs_frame *frames) {
  int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n) return;
  double p[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) p[i] = params[f * 16 + i];
  af_frame(p, frames + f);
}

// ---- Synthesizer::playTargetSequence (Synthesizer.cpp:1299-1422) ----------------------------

// OneDimAreaFunction::reset: the schwa init() latches (OneDimAreaFunction.cpp:281-350).
__constant__ double SCHWA[16] = {2.0, 1.0, 1.0, 3.02, 5.609, 1.0, 5.92, 2.879, 1.0, 8.48, 4.238, 1.0,
                                 15.31, 0.701, 16.44, 1.65};

// Lung pressure set by the fade-in statements (:1333-1346) at sample i < 0.1 fs.
__device__ double fade_in(const TargetPlan &t, int64_t i) {
  if (i < (double)0.05 * (double)t.fs) return 0.0;
  return t.P / 2 * cos((0.1 * t.fs - i) / (0.05 * t.fs) * PI) + t.P / 2;
}

// glottisParams[PRESSURE] after sample i's statements: fade-in, then held, then the
// fade-out of :1399-1403 with its denominator as written.
__device__ double lung_pressure(const TargetPlan &t, int64_t i) {
  double v;
  if (i < (double)0.1 * (double)t.fs) v = fade_in(t, i);
  else v = t.hold_j >= 0 ? fade_in(t, t.hold_j) : t.P;
  const double total = t.b[6];
  if (i > (double)(total - 0.1) * (double)t.fs)
    v = -t.P / 2 * cos((total * t.fs - i) / (total - 0.1 * t.fs) * PI) + t.P / 2;
  return v;
}

// F0 contour (:1348-1361).
__device__ double f0_contour(const TargetPlan &t, int64_t i) {
  const double *f = t.f0, *b = t.b, fs = t.fs;
  if (i < (double)b[1] * fs) return (f[0] + f[1]) / 2 + (f[1] - f[0]) / 2 * cos((b[1] * fs - i) / (b[1] * fs) * PI);
  if (i < (double)b[3] * fs)
    return (f[2] + f[1]) / 2 + (f[2] - f[1]) / 2 * cos((b[3] * fs - i) / ((b[3] - b[1]) * fs) * PI);
  return (f[3] + f[2]) / 2 + (f[3] - f[2]) / 2 * cos((b[6] * fs - i) / ((b[6] - b[3]) * fs) * PI);
}

// currentParams of sample i (:1364-1397) with interpolateParameters (:1286-1294).
__device__ void target_params(const double *s, const TargetPlan &t, int64_t i, double *p) {
  const double fs = t.fs, *b = t.b;
  int seg;  // 0..6: stationary 0, transition 0, stationary 1, ...
  if (i <= b[0] * fs) seg = 0;
  else if (i <= b[1] * fs) seg = 1;
  else if (i <= b[2] * fs) seg = 2;
  else if (i <= b[3] * fs) seg = 3;
  else if (i <= b[4] * fs) seg = 4;
  else if (i <= b[5] * fs) seg = 5;
  else seg = 6;
  const double *s0 = s + 16 * (seg / 2);
  if ((seg & 1) == 0) {
    for (int k = 0; k < 16; ++k) p[k] = s0[k];
  } else {
    const double *s1 = s0 + 16;
    const double t0 = b[seg - 1] * fs, t1 = b[seg] * fs;
    const double c = cos((t1 - i) / (t1 - t0) * PI);
    for (int k = 0; k < 16; ++k) p[k] = (s1[k] - s0[k]) / 2 * c + (s1[k] + s0[k]) / 2;
  }
}

__global__ void target_frames_kernel(const double *seq, int Q, TargetPlan t, int64_t k0, int n, int64_t fstride,
                                     afs_frame *frames) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)Q * n) return;
  const int q = (int)(idx / n), k = (int)(idx % n);
  const int64_t g = k0 + k;
  afs_frame *fr = frames + (int64_t)q * fstride + k;
  double p[16], gp[6];
  if (g == 0) {
    for (int i = 0; i < 16; ++i) p[i] = SCHWA[i];
    for (int i = 0; i < 6; ++i) gp[i] = t.glottis[i];
  } else {
    const int64_t i = g - 1;
    target_params(seq + (int64_t)q * 64, t, i, p);
    gp[0] = f0_contour(t, i);
    gp[1] = lung_pressure(t, i);
    for (int j = 2; j < 6; ++j) gp[j] = t.glottis[j];
  }
  af_frame(p, fr);
  fr->velum_opening_cm2 = 0.0;  // the Synthesizer's tube keeps Tube()'s closed velum
  for (int j = 0; j < 6; ++j) fr->glottis[j] = gp[j];
}

// The shape key of utterance u (shape_order, afs_capi.cpp), from its first frame: how narrow the
// tube is at its narrowest (in half-octave buckets of the area), then the noise class of its
// decisions (tree_plan.h plan_noise_class16: the synthesis kernel's noise-phase variant, the full
// phases first, so that a wave's four utterances share one variant), then where (section index),
// then the area itself (a float's bits: positive floats order as their bits).  Ascending, the
// narrowest constrictions -- the utterances with turbulence noise, the heaviest -- come first and
// alike shapes sit together.  (Measured against the section-major key: +0.8 % static vowels, equal
// on fricatives; descending: -1.3 %; profiles/r04v_shape_key_ab.txt.  The class as the first key
// instead of the second: within 0.2 %, profiles/r05g_class_key_ab.txt; no class key with the
// variants: -5 %, r05c_variants_ab.txt.)  A NaN area counts as wide.
__global__ void utterance_key_kernel(const afs_frame *frames, int64_t fstride, int B, uint64_t *keys, int noise_class) {
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= B) return;
  const afs_frame *f = frames + (int64_t)u * fstride;
  double amin = 1.0e30;
  int imin = 0;
  for (int m = 0; m < AFS_NUM_TUBE_SECTIONS; ++m) {
    const double a = f->area_cm2[m];
    if (a < amin) { amin = a; imin = m; }
  }
  const float af = amin > 0.0 ? (float)amin : 0.0f;
  const int bucket = (int)floorf(2.0f * log2f(af * 1000.0f + 1.0f));  // (0 .. ~28)
  tree::PlanKey k;
  double obst[4], po[4];
  plan_decide(tree::PlanGeomT<false>{f, f, 1.0, 0.0}, k, obst, po);  // (the first frame's decisions)
  const uint64_t cls = noise_class ? (uint64_t)tree::plan_noise_class16(tree::plan_key_noise(k), AFS_NZ_SET) : 0;
  keys[u] = noise_class == 2  // (the class after the narrowness bucket)
                ? ((uint64_t)bucket << 48) | (cls << 40) | ((uint64_t)imin << 32) | (uint64_t)__float_as_uint(af)
                : (cls << 48) | ((uint64_t)bucket << 40) | ((uint64_t)imin << 32) | (uint64_t)__float_as_uint(af);
}

// The slot order's rule on the device (afs_capi.cpp shape_order, one block): whether the call runs
// the noise-phase variants -- mode 2 always, 0 never, 1 when at least half the utterances have a light
// noise class (the class field at bit `shift` non-zero) or every SIMD runs many waves -- into
// *variants; without them the class field is masked out of the keys (it then plays no part in the
// order); idx[u] = u; the padding slots order[B .. slots) = B.
__global__ void __launch_bounds__(1024) order_rule_kernel(uint64_t *keys, int B, int shift, int mode, int many_waves,
                                                          int32_t *variants, int32_t *idx, int32_t *order, int slots) {
  __shared__ int light;
  if (threadIdx.x == 0) light = 0;
  __syncthreads();
  if (mode == 1 && shift >= 0) {
    int n = 0;
    for (int u = threadIdx.x; u < B; u += blockDim.x) n += ((keys[u] >> shift) & 3) != 0;
    atomicAdd(&light, n);
  }
  __syncthreads();
  const bool on = mode == 2 || (mode == 1 && (2 * (int64_t)light >= (int64_t)B || many_waves != 0));
  if (threadIdx.x == 0) *variants = on ? 1 : 0;
  const uint64_t mask = (shift >= 0 && !on) ? ~(3ull << shift) : ~0ull;
  for (int u = threadIdx.x; u < B; u += blockDim.x) {
    keys[u] &= mask;
    idx[u] = u;
  }
  for (int q = B + (int)threadIdx.x; q < slots; q += blockDim.x) order[q] = B;
}

}  // namespace

hipError_t launch_slot_order(uint64_t *keys, uint64_t *keys_sorted, int32_t *idx, int B, int shift, int mode,
                             bool many_waves, int32_t *variants, int32_t *order, int slots, void *temp,
                             size_t *temp_bytes, hipStream_t st) {
  if (!temp) return hipcub::DeviceRadixSort::SortPairs(nullptr, *temp_bytes, keys, keys_sorted, idx, order, B, 0, 64, st);
  hipLaunchKernelGGL(order_rule_kernel, dim3(1), dim3(1024), 0, st, keys, B, shift, mode, many_waves ? 1 : 0,
                     variants, idx, order, slots);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // stable (LSD radix): ties keep the utterance order, as the host's stable sort did
  return hipcub::DeviceRadixSort::SortPairs(temp, *temp_bytes, keys, keys_sorted, idx, order, B, 0, 64, st);
}

hipError_t launch_utterance_keys(const afs_frame *frames, int64_t fstride, int B, uint64_t *keys, int noise_class,
                                 hipStream_t st) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(utterance_key_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st, frames, fstride, B,
                     keys, noise_class);
  return hipGetLastError();
}

hipError_t launch_af_to_frames(const double *params, int64_t n, afs_frame *frames, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(af_to_frames_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, params, n, frames);
  return hipGetLastError();
}

hipError_t launch_target_frames(const double *seq, int Q, const TargetPlan &plan, int64_t k0, int n,
                                int64_t fstride, afs_frame *frames, hipStream_t st) {
  const int64_t total = (int64_t)Q * n;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(target_frames_kernel, dim3((unsigned)((total + 63) / 64)), dim3(64), 0, st, seq, Q, plan, k0,
                     n, fstride, frames);
  return hipGetLastError();
}

}  // namespace afs
