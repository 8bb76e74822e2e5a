// Development probe (not part of libafs): accuracy of v_rcp_f64 / v_sqrt_f64 / v_rsq_f64
// with 0, 1 or 2 Newton steps against IEEE division / sqrt, and the dependent-chain latency
// of a few fp64 instructions for one wave per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o f64_ops f64_ops.hip && ./f64_ops
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

__device__ double rcp_n(double d, int n) {
  double r = __builtin_amdgcn_rcp(d);
  for (int i = 0; i < n; ++i) {
    double e = fma(-d, r, 1.0);
    r = fma(r, e, r);
  }
  return r;
}

// sqrt of a positive, finite, normal x >= 2^-767: LLVM's f64 sqrt sequence without the
// range scaling and the zero/infinity fix-up (tree_core.h fast_sqrt)
__device__ double sqrt_noscale(double x) {
  double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  double d = fma(-g, g, x);
  g = fma(d, h, g);
  d = fma(-g, g, x);
  return fma(d, h, g);
}

__global__ void sqrt_cmp(const double *x, int n, unsigned long long *bad) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (__double_as_longlong(sqrt(x[i])) != __double_as_longlong(sqrt_noscale(x[i]))) atomicAdd(bad, 1ull);
}

__global__ void accuracy(const double *x, int n, double *out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double d = x[i];
  out[8 * i + 0] = 1.0 / d;
  out[8 * i + 1] = rcp_n(d, 0);
  out[8 * i + 2] = rcp_n(d, 1);
  out[8 * i + 3] = rcp_n(d, 2);
  out[8 * i + 4] = sqrt(d);
  out[8 * i + 5] = __builtin_amdgcn_sqrt(d);
  out[8 * i + 6] = __builtin_amdgcn_rsq(d);
  out[8 * i + 7] = 1.0 / sqrt(d);
}

// dependent chains of `reps` operations; one wave per block, one block per CU
template <int OP>
__global__ void chain(double *io, int reps, long long *cyc) {
  double a = io[threadIdx.x], b = io[64 + threadIdx.x];
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < reps; ++k) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (OP == 0) a = a * b;                       // v_mul_f64
      if (OP == 1) a = fma(a, b, b);                // v_fma_f64
      if (OP == 2) a = __builtin_amdgcn_rcp(a);     // v_rcp_f64
      if (OP == 3) a = sqrt(a);                     // libm sqrt (IEEE sequence)
      if (OP == 4) a = __builtin_amdgcn_sqrt(a);    // v_sqrt_f64
      if (OP == 5) a = a / b;                       // IEEE division sequence
      if (OP == 6) a = a + b;                       // v_add_f64
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  io[threadIdx.x] = a;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

static double ulps(double got, double ref) {
  if (got == ref) return 0.0;
  int64_t a, b;
  std::memcpy(&a, &got, 8);
  std::memcpy(&b, &ref, 8);
  return std::fabs((double)(a - b));
}

template <int OP>
static int run_chain(const char *name, double *d_io, long long *d_cyc) {
  const int reps = 256;
  hipLaunchKernelGGL(chain<OP>, dim3(256), dim3(64), 0, nullptr, d_io, reps, d_cyc);
  CK(hipDeviceSynchronize());
  std::vector<long long> c(256);
  CK(hipMemcpy(c.data(), d_cyc, 256 * sizeof(long long), hipMemcpyDeviceToHost));
  double s = 0;
  for (long long v : c) s += (double)v;
  printf("  %-28s %7.2f cycles per dependent op\n", name, s / 256 / (reps * 16.0));
  return 0;
}

int main() {
  const int n = 1 << 20;
  std::vector<double> x(n);
  uint64_t st = 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < n; ++i) {
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    double m = 1.0 + (double)(st >> 11) * (1.0 / 9007199254740992.0);  // [1, 2)
    int e = (int)((st >> 3) % 80) - 40;
    x[i] = std::ldexp(m, e);
  }
  double *dx, *dout;
  CK(hipMalloc(&dx, n * sizeof(double)));
  CK(hipMalloc(&dout, 8 * (size_t)n * sizeof(double)));
  CK(hipMemcpy(dx, x.data(), n * sizeof(double), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(accuracy, dim3(n / 256), dim3(256), 0, nullptr, dx, n, dout);
  CK(hipDeviceSynchronize());
  std::vector<double> o(8 * (size_t)n);
  CK(hipMemcpy(o.data(), dout, o.size() * sizeof(double), hipMemcpyDeviceToHost));
  double mx[8] = {0};
  long exact[8] = {0};
  for (int i = 0; i < n; ++i) {
    const double rr = 1.0 / x[i], sq = std::sqrt(x[i]), rs = 1.0 / std::sqrt(x[i]);
    const double ref[8] = {rr, rr, rr, rr, sq, sq, rs, rs};
    for (int k = 0; k < 8; ++k) {
      double u = ulps(o[8 * (size_t)i + k], ref[k]);
      if (u > mx[k]) mx[k] = u;
      if (u == 0) exact[k]++;
    }
  }
  const char *names[8] = {"1.0/d (device IEEE div)", "v_rcp_f64", "v_rcp_f64 + 1 Newton", "v_rcp_f64 + 2 Newton",
                          "sqrt (device)", "v_sqrt_f64", "v_rsq_f64 vs 1/sqrt", "1.0/sqrt(d) device"};
  printf("accuracy vs host IEEE (%d inputs, 2^-40..2^40): max ulps / exactly rounded fraction\n", n);
  for (int k = 0; k < 8; ++k) printf("  %-28s %10.0f  %.4f\n", names[k], mx[k], (double)exact[k] / n);
  {
    unsigned long long *dbad, bad = 0;
    CK(hipMalloc(&dbad, 8));
    CK(hipMemcpy(dbad, &bad, 8, hipMemcpyHostToDevice));
    long tested = 0;
    for (int range = 0; range < 3; ++range) {  // 2^-40..2^40 (above), then wide / narrow exponents
      if (range > 0) {
        for (int i = 0; i < n; ++i) {
          st ^= st << 13; st ^= st >> 7; st ^= st << 17;
          double m = 1.0 + (double)(st >> 11) * (1.0 / 9007199254740992.0);
          int e = range == 1 ? (int)((st >> 3) % 1400) - 700 : (int)((st >> 3) % 60) - 30;
          x[i] = std::ldexp(m, e);
        }
        CK(hipMemcpy(dx, x.data(), n * sizeof(double), hipMemcpyHostToDevice));
      }
      hipLaunchKernelGGL(sqrt_cmp, dim3(n / 256), dim3(256), 0, nullptr, dx, n, dbad);
      CK(hipDeviceSynchronize());
      tested += n;
    }
    CK(hipMemcpy(&bad, dbad, 8, hipMemcpyDeviceToHost));
    printf("sqrt without range scaling vs device sqrt: %llu of %ld inputs differ (2^-700..2^700)\n", bad, tested);
  }
  double *dio;
  long long *dcyc;
  std::vector<double> io(128, 1.0000001);
  CK(hipMalloc(&dio, 128 * sizeof(double)));
  CK(hipMalloc(&dcyc, 256 * sizeof(long long)));
  CK(hipMemcpy(dio, io.data(), 128 * sizeof(double), hipMemcpyHostToDevice));
  printf("dependent-chain latency, one wave per CU (s_memtime cycles):\n");
  run_chain<0>("v_mul_f64", dio, dcyc);
  run_chain<6>("v_add_f64", dio, dcyc);
  run_chain<1>("v_fma_f64", dio, dcyc);
  run_chain<2>("v_rcp_f64", dio, dcyc);
  run_chain<4>("v_sqrt_f64", dio, dcyc);
  run_chain<3>("sqrt (IEEE sequence)", dio, dcyc);
  run_chain<5>("a / b (IEEE sequence)", dio, dcyc);
  return 0;
}
