// pair_emu.cpp -- TEST-ONLY host execution of the wave-pair step (tree_core.h sample_step_pair,
// compiled with AFS_PAIR=1): the DYN and the STAT role of one utterance run on two threads that meet
// at the step's workgroup barriers (x.bar()), each over its own lane array, both on one LDS block --
// the decomposition tree_kernel.h tree_pair_run runs on two waves.  tests/test_tree_emu.py checks it
// against the one-wave step (tree_emu.cpp, tone filter in K6 as on the device) bit for bit.  Never
// part of the product.
#include <thread>
#include <vector>

#include "tree_core.h"

using namespace afs;
using namespace afs::tree;

#include "cpu_exec.h"

static_assert(AFS_PAIR, "build with -DAFS_PAIR=1");

namespace {

template <int W, int MODEL>
long run_pair(const afs_frame *frames, int F, int hop, unsigned seed, double fs, const afs_options &opt,
              double *out, uint64_t *draws) {
  std::vector<Tables> tab(1);
  Tables &T = tab[0];
  build_tables(&T, fs, opt);
  if (T.n_rounds < 0) return -1;
  std::vector<Lane<W>> RD(W), RS(W);
  for (int gl = 0; gl < W; ++gl) {
    reset_lane<W>(gl, RD[gl]);
    reset_lane<W>(gl, RS[gl]);
  }
  std::vector<double> X(X_TOTAL);
  reset_lds(X.data(), seed);
  {  // (tree_pair_run: the STAT wave puts the rand() ring's head and pending count into LDS)
    int32_t *hp = (int32_t *)(X.data() + X_RNGHP);
    hp[0] = RS[0].rhead;
    hp[1] = RS[0].rpend;
  }
  Barrier2 bar;
  CpuExec<W, true> exD{RD.data(), &bar}, exS{RS.data(), &bar};
  const long total = (long)(F - 1) * hop;
  std::vector<double> flow(total), p25(total);
  const bool two = opt.glottis_model == AFS_GLOTTIS_TWO_MASS;
  auto dyn = [&] {
    long t = 0;
    for (int k = 1; k < F; ++k) {
      for (int gl = 0; gl < W; ++gl) frame_load<W>(gl, RD[gl], X.data(), frames + k - 1, frames + k);
      exD.bar();  // (the hop's frames in LDS for both roles)
      for (int i = 0; i < hop; ++i, ++t) {
        const double ratio = (double)i / (double)hop;
        sample_step_pair<W, MODEL, NZ_FULL, ROLE_DYN>(exD, X.data(), T.uni, T.consts, ratio, (int)(t & 1));
        flow[t] = RD[0].sample;
        p25[t] = RD[2].p[0];  // (section 25: lane 2's dynamic slot 0)
      }
    }
  };
  auto stat = [&] {
    long t = 0;
    for (int k = 1; k < F; ++k) {
      exS.bar();
      for (int i = 0; i < hop; ++i, ++t) {
        const double ratio = (double)i / (double)hop;
        uint64_t w[PLAN_WORDS];  // (K5's record of the sample: the STAT wave holds the plan words)
        plan_sample(frames + k - 1, frames + k, ratio, T.consts.sec, two, w);
        for (int gl = 0; gl < W; ++gl) RS[gl].planw = w[gl % PLAN_WORDS];
        sample_step_pair<W, MODEL, NZ_FULL, ROLE_STAT>(exS, X.data(), T.uni, T.consts, ratio, (int)(t & 1));
      }
    }
  };
  std::thread th(stat);
  dyn();
  th.join();
  // K6 (tree_output_kernel) per hop, its filter state in the LDS block, which the step leaves alone
  for (long t0 = 0; t0 < total; t0 += hop) {
    for (int i = 0; i < hop; ++i) out[t0 + i] = flow[t0 + i];
    if (opt.radiation_from_skin) tone_output_run(X.data(), T.consts, p25.data() + t0, out + t0, hop);
    else output_filter_run(X.data(), T.consts, out + t0, hop);
  }
  *draws = *(const uint64_t *)(X.data() + X_NDRAW);
  return total;
}

template <int W>
long run_w(const afs_frame *frames, int F, int hop, unsigned seed, double fs, const afs_options &opt, double *out,
           uint64_t *draws) {
  if (opt.glottis_model == AFS_GLOTTIS_TWO_MASS)
    return run_pair<W, AFS_GLOTTIS_TWO_MASS>(frames, F, hop, seed, fs, opt, out, draws);
  return run_pair<W, AFS_GLOTTIS_TRIANGULAR>(frames, F, hop, seed, fs, opt, out, draws);
}

}  // namespace

// options as emu_tree_utterance_opt (tree_emu.cpp); W: 16 (the throughput pairs) or 64 (the voice pairs)
extern "C" long emu_pair_utterance(const afs_frame *frames, int F, int hop, unsigned seed, double fs, int W,
                                   const int *iopt, double ratio, double *out, uint64_t *draws) {
  afs_options opt = afs::default_options();
  if (iopt) {
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
  }
  if (W == 16) return run_w<16>(frames, F, hop, seed, fs, opt, out, draws);
  if (W == 64) return run_w<64>(frames, F, hop, seed, fs, opt, out, draws);
  return -2;
}
