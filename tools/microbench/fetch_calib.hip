// Development probe (not part of libafs): FETCH_SIZE calibration for the read patterns of the
// synthesis kernel (MI355X_MICROARCH.md, HBM: "other access widths are uncalibrated").  Each
// kernel reads a 2 GiB buffer once (8x the 256 MiB Infinity Cache); rocprofv3 --pmc FETCH_SIZE
// then gives KiB per dispatch against the 2 GiB read.
//   hipcc --offload-arch=gfx950 -O3 -o fetch_calib fetch_calib.hip
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d OUT -o run -- ./fetch_calib
// Patterns:
//   b64_row16  16 lanes read the 16 u64 of one 128-B record (the plan read, tree_kernel.h)
//   b128       16 B per lane, fully coalesced (the guide's calibrated case)
//   b64_lane0  one lane in 16 reads 8 B, consecutive (lane 0's frame / flow reads)
//   rec1072    each lane walks its own 1072-B record with 8-B loads (K5's interval kernel)
//   row8       each lane reads its own row, 8 doubles per step as 16-B loads (K6)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

constexpr size_t BYTES = (size_t)2 << 30;

__global__ void b64_row16(const uint64_t *p, size_t n, uint64_t *sink) {
  uint64_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc += p[i];
  if (acc == 0x123456789ull) sink[0] = acc;
}

__global__ void b128(const ulonglong2 *p, size_t n, uint64_t *sink) {
  uint64_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const ulonglong2 v = p[i];
    acc += v.x ^ v.y;
  }
  if (acc == 0x123456789ull) sink[0] = acc;
}

// one lane of each 16 reads: u64 index = thread / 16 * 16 .. (the lane-0 pattern reads 8 of
// every 128 bytes; 1/16 of the buffer)
__global__ void b64_lane0(const uint64_t *p, size_t n, uint64_t *sink) {
  uint64_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    if ((threadIdx.x & 15) == 0) acc += p[i];
  if (acc == 0x123456789ull) sink[0] = acc;
}

// K5's interval kernel (tds_plan.hip plan_hop_iv_kernel): each thread walks its own 1072-B frame
// record field by field (8-B loads; the lanes of a wave 1072 B apart)
__global__ void rec1072(const uint64_t *p, size_t nrec, uint64_t *sink) {
  uint64_t acc = 0;
  for (size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x; r < nrec; r += (size_t)gridDim.x * blockDim.x)
    for (int m = 0; m < 134; ++m) acc += p[r * 134 + m];
  if (acc == 0x123456789ull) sink[0] = acc;
}

// K6 (tds_tree.hip tree_output_kernel): one thread per utterance row, 8 consecutive doubles per
// step as four 16-B loads (the lanes of a wave one row apart)
__global__ void row8(const ulonglong2 *p, size_t rows, size_t row_u128, uint64_t *sink) {
  uint64_t acc = 0;
  const size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < rows)
    for (size_t i = 0; i < row_u128; i += 4) {
      const ulonglong2 *q = p + r * row_u128 + i;
      const ulonglong2 a = q[0], b = q[1], c = q[2], d = q[3];
      acc += a.x ^ b.y ^ c.x ^ d.y;
    }
  if (acc == 0x123456789ull) sink[0] = acc;
}

int main() {
  uint64_t *buf = nullptr, *sink = nullptr;
  CK(hipMalloc(&buf, BYTES));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(buf, 1, BYTES));
  const dim3 grid(256 * 8 * 4), block(256);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(b64_row16, grid, block, 0, 0, buf, BYTES / 8, sink);
    hipLaunchKernelGGL(b128, grid, block, 0, 0, (const ulonglong2 *)buf, BYTES / 16, sink);
    hipLaunchKernelGGL(b64_lane0, grid, block, 0, 0, buf, BYTES / 8, sink);
    hipLaunchKernelGGL(rec1072, grid, block, 0, 0, buf, BYTES / 1072, sink);
    hipLaunchKernelGGL(row8, dim3(8192 / 64), dim3(64), 0, 0, (const ulonglong2 *)buf, (size_t)8192,
                       BYTES / 16 / 8192, sink);
  }
  CK(hipDeviceSynchronize());
  printf("read bytes per dispatch: b64_row16 %zu, b128 %zu, b64_lane0 %zu (8 B of every 128), rec1072 %zu, row8 %zu\n",
         BYTES, BYTES, BYTES / 16, BYTES / 1072 * 1072, BYTES);
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
