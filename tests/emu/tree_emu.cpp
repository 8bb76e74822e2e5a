// tree_emu.cpp -- TEST-ONLY host execution of the cooperative tree kernel's phase code.
//
// Runs csrc/tree_core.h's sample_step with the W lanes of each phase executed one after
// another (phases only read LDS data written by earlier phases, so this is the same
// computation the GPU does in lock step).  Used by tests/test_tree_emu.py to check the
// decomposition (slot ownership, LDS exchange, the tree LDL^T schedule) against the
// oracle on the CPU.  Never part of the product; libafs.so does not contain it.
#include <cstring>
#include <vector>

#include "tree_core.h"

using namespace afs;
using namespace afs::tree;

#include "cpu_exec.h"

namespace {

// Hop mode (tree_plan.h PlanHop): hops >= PLAN_HOP_MIN take their plan words from the hop
// record (plan_hop_host, as K5 builds it) evaluated per sample (plan_word_fast, as the synthesis
// kernel), mixed hops from the dense records.  Off by default (dense records at every hop).
int g_hop_mode = 0;
long g_hops = 0, g_mixed_hops = 0;
// Tone-in-K6 mode (the device default): the sample step leaves out the glottal-tone filter, lane
// 2's slot 0 (section 25's new pressure) is stored per sample, and tone_output_run adds the tone to the
// hop's flows before the output filter -- as tree_kernel.h + tree_output_kernel.  Off by default.
int g_tone_k6 = 0;
// Noise-phase variants (the device's hop-mode default, tree_kernel.h noise_variant): each hop runs
// in the lightest variant (tree_core.h NoiseV) that serves its record's noise mask and the dipole
// slots still holding amplitude, the hop playing the part of a launch.  Off by default; counts of
// the hops run in each variant since the last emu_tree_variant_counts.
int g_noise_variants = 0;
long g_variant_hops[NZ_COUNT] = {};

template <int W>
int emu_noise_variant(uint64_t m, const Lane<W> *R) {
  for (int gl = 0; gl < W; ++gl)
    for (int k = 0; k < Shape<W>::NDP; ++k)
      if (R[gl].damp[k] != 0.0 && gl + k * W < NDIP) m |= 1ull << (gl + k * W);
  int nz = NZ_FULL;
  if ((m & ~NoiseV<W, NZ_T1ALL>::SERVES) == 0) nz = NZ_T1ALL;  // (every variant is emulated)
  if ((m & ~NoiseV<W, NZ_TONGUE1>::SERVES) == 0) nz = NZ_TONGUE1;
  if ((m & ~NoiseV<W, NZ_GLOTTIS>::SERVES) == 0) nz = NZ_GLOTTIS;
  return nz;
}

// (variants on: the device's arrangement, the variant switched at run time in the phase after the
// geometry / network block, NZ_DYN; off: the full phases with the targets inside the block)
template <int W, int MODEL, class Xc>
void step_nz(int nz, Xc &ex, double *X, const Tables &T, double ratio, bool defer) {
  if (g_noise_variants) sample_step<W, MODEL, NZ_DYN>(ex, X, T.uni, T.consts, ratio, defer, nz);
  else sample_step<W, MODEL, NZ_FULL>(ex, X, T.uni, T.consts, ratio, defer);
}

template <int W, bool TONE>
long run_impl(const afs_frame *frames, int F, int hop, unsigned seed, double fs, const afs_options &opt,
         double *out, double *dump_p, double *dump_u, int ndump) {
  static Tables T;
  build_tables(&T, fs, opt);
  if (T.n_rounds < 0) return -1;
  std::vector<Lane<W>> R(W);
  std::vector<double> X(X_TOTAL);
  for (int gl = 0; gl < W; ++gl) reset_lane<W>(gl, R[gl]);
  reset_lds(X.data(), seed);
  CpuExec<W, TONE> ex{R.data()};
  long t = 0;
  // as the GPU kernel (tree_kernel.h): the tone-in-K6 build always defers the output filter
  const bool defer = TONE || hop >= OUT_DEFER_MIN_HOP;
  std::vector<double> p25(TONE ? hop : 0);
  const bool two = opt.glottis_model == AFS_GLOTTIS_TWO_MASS;
  const bool hops = g_hop_mode && hop >= PLAN_HOP_MIN;
  for (int k = 1; k < F; ++k) {
    for (int gl = 0; gl < W; ++gl) frame_load<W>(gl, R[gl], X.data(), frames + k - 1, frames + k);
    PlanHop H{};
    if (hops) {
      plan_hop_host(frames + k - 1, frames + k, hop, 0, hop, T.consts.sec, two, H);
      ++g_hops;
      g_mixed_hops += H.mixed ? 1 : 0;
    }
    const long t0 = t;
    const int nz = (hops && g_noise_variants) ? emu_noise_variant<W>(H.noise, R.data()) : (int)NZ_FULL;
    if (hops && g_noise_variants) ++g_variant_hops[nz];
    for (int i = 0; i < hop; ++i) {
      double ratio = (double)i / (double)hop;
      uint64_t w[PLAN_WORDS];  // K5's record of this sample (tree_plan.h)
      if (hops && !H.mixed)
        for (int q = 0; q < PLAN_WORDS; ++q) w[q] = plan_word_fast(H.kind[q], H.p[q], ratio);
      else
        plan_sample(frames + k - 1, frames + k, ratio, T.consts.sec, two, w);
      for (int gl = 0; gl < W; ++gl) R[gl].planw = w[gl % PLAN_WORDS];
      if (opt.glottis_model == AFS_GLOTTIS_TWO_MASS)
        step_nz<W, AFS_GLOTTIS_TWO_MASS>(nz, ex, X.data(), T, ratio, defer);
      else
        step_nz<W, AFS_GLOTTIS_TRIANGULAR>(nz, ex, X.data(), T, ratio, defer);
      out[t] = R[0].sample;
      if constexpr (TONE) p25[i] = R[2].p[0];
      if (t < ndump) {
        for (int gl = 0; gl < W; ++gl)
          for (int j = 0; j < Shape<W>::NSL; ++j) {
            int s = slot_section<W>(j, gl);
            if (s >= 0) dump_p[t * NS + s] = R[gl].p[j];
          }
        for (int c = 0; c < NC; ++c) dump_u[t * NC + c] = X[X_U + c];
      }
      ++t;
    }
    if (TONE && opt.radiation_from_skin) tone_output_run(X.data(), T.consts, p25.data(), out + t0, hop);
    else if (defer) output_filter_run(X.data(), T.consts, out + t0, hop);
  }
  return t;
}

template <int W>
long run(const afs_frame *frames, int F, int hop, unsigned seed, double fs, const afs_options &opt,
         double *out, double *dump_p, double *dump_u, int ndump) {
  return g_tone_k6 ? run_impl<W, true>(frames, F, hop, seed, fs, opt, out, dump_p, dump_u, ndump)
                   : run_impl<W, false>(frames, F, hop, seed, fs, opt, out, dump_p, dump_u, ndump);
}

}  // namespace

extern "C" long emu_tree_utterance(const afs_frame *frames, int F, int hop, unsigned seed, double fs, int W,
                                   double *out, double *dump_p, double *dump_u, int ndump) {
  afs_options opt = afs::default_options();
  switch (W) {
    case 16: return run<16>(frames, F, hop, seed, fs, opt, out, dump_p, dump_u, ndump);
    case 32: return run<32>(frames, F, hop, seed, fs, opt, out, dump_p, dump_u, ndump);
    case 64: return run<64>(frames, F, hop, seed, fs, opt, out, dump_p, dump_u, ndump);
  }
  return -2;
}

// options: turbulence, soft walls, noise, skin radiation, fossa, inner length corrections,
// transvelar coupling, glottis loss (ints) and the flow-separation area ratio.
extern "C" long emu_tree_utterance_opt(const afs_frame *frames, int F, int hop, unsigned seed, double fs,
                                       const int *iopt, double ratio, double *out) {
  afs_options opt = afs::default_options();
  opt.turbulence_losses = iopt[0];
  opt.soft_walls = iopt[1];
  opt.generate_noise_sources = iopt[2];
  opt.radiation_from_skin = iopt[3];
  opt.piriform_fossa = iopt[4];
  opt.inner_length_corrections = iopt[5];
  opt.transvelar_coupling = iopt[6];
  opt.glottis_loss = iopt[7];
  opt.glottis_model = iopt[8];
  opt.flow_separation_area_ratio = ratio;
  return run<16>(frames, F, hop, seed, fs, opt, out, nullptr, nullptr, 0);
}

extern "C" void emu_tree_set_hop_mode(int on) { g_hop_mode = on; }
extern "C" void emu_tree_set_tone_k6(int on) { g_tone_k6 = on; }
extern "C" void emu_tree_set_noise_variants(int on) { g_noise_variants = on; }
// hops run in each noise-phase variant (NZ_FULL, NZ_T1ALL, NZ_TONGUE1, NZ_GLOTTIS) since the last call
extern "C" void emu_tree_variant_counts(long *counts) {
  for (int v = 0; v < NZ_COUNT; ++v) {
    counts[v] = g_variant_hops[v];
    g_variant_hops[v] = 0;
  }
}
// hops run in hop mode since the last call, and how many of them were mixed
extern "C" void emu_tree_hop_counts(long *hops, long *mixed) {
  *hops = g_hops;
  *mixed = g_mixed_hops;
  g_hops = g_mixed_hops = 0;
}

extern "C" int emu_tree_rounds(double fs) {
  static Tables T;
  afs_options opt = afs::default_options();
  build_tables(&T, fs, opt);
  return T.n_rounds;
}
