// cse_pow_repro.hip -- minimal reproducer: device pow / exp / log10 of double built with and
// without `-mllvm -disable-machine-cse` (development tool, not product).
//   hipcc --offload-arch=gfx950 -O3 cse_pow_repro.hip -o cse_default
//   hipcc --offload-arch=gfx950 -O3 -mllvm -disable-machine-cse cse_pow_repro.hip -o cse_off
// Each binary evaluates pow(10, x / 20), pow(x, 1.5), exp(x / 20) and log10(|x| + 1) for x in
// [-60, 20] on the GPU and prints the largest distance in ulps from the host's libm.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void k(const double *x, double *out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double v = x[i];
  out[4 * i + 0] = pow(10.0, v / 20.0);
  out[4 * i + 1] = pow(fabs(v) + 0.5, 1.5);
  out[4 * i + 2] = exp(v / 20.0);
  out[4 * i + 3] = log10(fabs(v) + 1.0);
}

static int64_t ulps(double a, double b) {
  int64_t ia, ib;
  std::memcpy(&ia, &a, 8);
  std::memcpy(&ib, &b, 8);
  return ia > ib ? ia - ib : ib - ia;
}

int main() {
  const int n = 1 << 16;
  std::vector<double> x(n), out(4 * n);
  for (int i = 0; i < n; ++i) x[i] = -60.0 + 80.0 * i / n;
  double *dx, *dout;
  if (hipMalloc(&dx, n * 8) != hipSuccess || hipMalloc(&dout, 4 * n * 8) != hipSuccess) return 1;
  (void)hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dx, dout, n);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  (void)hipMemcpy(out.data(), dout, 4 * n * 8, hipMemcpyDeviceToHost);
  const char *name[4] = {"pow(10, x/20)", "pow(|x|+0.5, 1.5)", "exp(x/20)", "log10(|x|+1)"};
  for (int f = 0; f < 4; ++f) {
    int64_t worst = 0;
    int at = 0;
    for (int i = 0; i < n; ++i) {
      const double v = x[i];
      const double h = f == 0 ? std::pow(10.0, v / 20.0)
                     : f == 1 ? std::pow(std::fabs(v) + 0.5, 1.5)
                     : f == 2 ? std::exp(v / 20.0)
                              : std::log10(std::fabs(v) + 1.0);
      const int64_t u = ulps(out[4 * i + f], h);
      if (u > worst) { worst = u; at = i; }
    }
    std::printf("%-18s max %lld ulps (x = %.6f: gpu %.17g host %.17g)\n", name[f], (long long)worst, x[at],
                out[4 * at + f], f == 0 ? std::pow(10.0, x[at] / 20.0) : f == 1 ? std::pow(std::fabs(x[at]) + 0.5, 1.5)
                : f == 2 ? std::exp(x[at] / 20.0) : std::log10(std::fabs(x[at]) + 1.0));
  }
  (void)hipFree(dx);
  (void)hipFree(dout);
  return 0;
}
