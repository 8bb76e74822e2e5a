// tds_plan.hip -- the noise-source plan kernel (K5): the constriction scans of every sample
// ahead of the time loop (tree_plan.h), one thread per (frame row, sample).  A file of its own
// so that it is compiled with its own flags (build.py).
#include "afs_tree.h"
#include "tree_plan.h"

namespace afs {

using namespace tree;

namespace {

// Grid (rows, sample blocks of PLAN_BLOCK): one thread per (frame row, sample), a block of
// consecutive samples of one row.  When the block's samples span at most PLAN_STAGE frames
// (hops >= 128), the frames are staged in LDS first: the plan's scans read every section's
// area / length / articulator several times, and from LDS those reads cost a fraction of the
// cache-hit latency of global loads.  Shorter hops (target sequences, hop 1) read the frames
// from global memory.  Each thread stores its own 128-B record with eight 16-byte stores (the
// block's records are contiguous; L2 merges the partial lines): no LDS for the records, so a K5
// block (4.3 KB of LDS, 80 VGPRs) fits on a CU beside the synthesis kernel's block, which K5 of
// the next launch runs concurrently with (afs_capi.cpp run_chunks).  Assembling the records in
// LDS first for one coalesced store per lane and step measured within 2 %.
#ifndef AFS_PLAN_BLOCK
#define AFS_PLAN_BLOCK 256
#endif
constexpr int PLAN_BLOCK = AFS_PLAN_BLOCK, PLAN_STAGE = 4;
constexpr int FRAME_WORDS = (int)(sizeof(afs_frame) / 8);
static_assert(sizeof(afs_frame) % 8 == 0, "frames are copied as 8-byte words");

__global__ void __launch_bounds__(PLAN_BLOCK) plan_kernel(PlanArgs a) {
  __shared__ uint64_t fr_lds[PLAN_STAGE][FRAME_WORDS];
  const int64_t n = a.s_end - a.s_begin;
  const int64_t row = blockIdx.x;
  const int64_t t_first = (int64_t)blockIdx.y * PLAN_BLOCK;
  const int64_t t_last = (t_first + PLAN_BLOCK < n ? t_first + PLAN_BLOCK : n) - 1;
  const int64_t t = t_first + threadIdx.x;
  const afs_frame *f = a.frames + row * a.frame_stride;
  // sample s plays frames s / hop and s / hop + 1
  const int64_t k_lo = (a.s_begin + t_first) / a.hop, k_hi = (a.s_begin + t_last) / a.hop + 1;
  const bool staged = k_hi - k_lo + 1 <= PLAN_STAGE;  // uniform over the block
  if (staged) {
    const uint64_t *src = (const uint64_t *)(f + k_lo);
    const int words = (int)(k_hi - k_lo + 1) * FRAME_WORDS;
    for (int w = threadIdx.x; w < words; w += PLAN_BLOCK) (&fr_lds[0][0])[w] = src[w];
    __syncthreads();
    // the areas clamped once per frame (Tube::setPharynxMouthGeometry's MIN_AREA, idempotent)
    // instead of twice per sample and section
    for (int q = threadIdx.x; q < (int)(k_hi - k_lo + 1) * NPM; q += PLAN_BLOCK) {
      double *ar = ((afs_frame *)fr_lds[q / NPM])->area_cm2 + q % NPM;
      *ar = plan_clampA(*ar);
    }
    __syncthreads();
  }
  if (t < n) {
    const int64_t s = a.s_begin + t;
    const int64_t k = s / a.hop + 1;
    const int i = (int)(s - (k - 1) * a.hop);
    const double ratio = (double)i / (double)a.hop;
    uint64_t w[PLAN_WORDS];
    // two instantiations of the scans: LDS frames (ds_read) and global frames (global loads);
    // one pointer that may point at either would make every frame read a flat load
    if (staged)
      plan_sample<true>((const afs_frame *)fr_lds[k - 1 - k_lo], (const afs_frame *)fr_lds[k - k_lo], ratio, a.uo,
                        a.two_mass != 0, w);
    else
      plan_sample(f + (k - 1), f + k, ratio, a.uo, a.two_mass != 0, w);
    ulonglong2 *o = (ulonglong2 *)(a.plan + (row * a.plan_stride + t) * PLAN_WORDS);
#pragma unroll
    for (int q = 0; q < PLAN_WORDS / 2; ++q) o[q] = make_ulonglong2(w[2 * q], w[2 * q + 1]);
  }
}

}  // namespace

hipError_t launch_plan(const PlanArgs &a, hipStream_t st) {
  const int64_t n = a.s_end - a.s_begin;
  if (n <= 0 || a.rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(plan_kernel, dim3((unsigned)a.rows, (unsigned)((n + PLAN_BLOCK - 1) / PLAN_BLOCK)),
                     dim3(PLAN_BLOCK), 0, st, a);
  return hipGetLastError();
}

}  // namespace afs
