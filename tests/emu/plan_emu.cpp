// plan_emu.cpp -- TEST-ONLY host evaluation of the noise-source plan (csrc/tree_plan.h): the
// dense records plan_sample computes (as K5 does), the hop records plan_hop_host builds (as K5's
// hop mode does), the interval decisions and the host form of the synthesis kernel's per-sample
// word evaluation.  tests/test_plan_gpu.py and tests/test_plan_hops.py compare K5 and the
// synthesis kernel with these.  Never part of the product; libafs.so does not contain it.
#include <cstring>
#include <vector>

#include "tree_core.h"

using namespace afs;

// The noise-source plan records (tree_plan.h plan_sample, as K5 evaluates them) of samples
// [s0, s1) of frames[rows][F] at this hop: out[rows][s1 - s0][PLAN_WORDS].
extern "C" int emu_plan_records(const afs_frame *frames, int rows, int F, int hop, long s0, long s1, double fs,
                                int two_mass, uint64_t *out) {
  static Tables T;
  afs_options opt = afs::default_options();
  opt.glottis_model = two_mass ? AFS_GLOTTIS_TWO_MASS : AFS_GLOTTIS_TRIANGULAR;
  build_tables(&T, fs, opt);
  const SecRec *uo = T.consts.sec;
  for (int r = 0; r < rows; ++r)
    for (long s = s0; s < s1; ++s) {
      const long k = s / hop + 1;
      const int i = (int)(s - (k - 1) * hop);
      const double ratio = (double)i / (double)hop;
      const afs_frame *f = frames + (long)r * F;
      tree::plan_sample(f + k - 1, f + k, ratio, uo, two_mass != 0,
                        out + ((long)r * (s1 - s0) + (s - s0)) * tree::PLAN_WORDS);
    }
  return 0;
}

// The hop records (tree_plan.h plan_hop_host, as K5's hop mode builds them) of the hops that
// samples [s0, s1) of frames[rows][F] span at this hop (>= PLAN_HOP_MIN), with the tree
// kernel's LDS offsets: out[rows][plan_hop_slots(s0, s1, hop)] PlanHop records.
extern "C" int emu_plan_hops(const afs_frame *frames, int rows, int F, int hop, long s0, long s1, double fs,
                             int two_mass, tree::PlanHop *out) {
  static Tables T;
  afs_options opt = afs::default_options();
  opt.glottis_model = two_mass ? AFS_GLOTTIS_TWO_MASS : AFS_GLOTTIS_TRIANGULAR;
  build_tables(&T, fs, opt);
  const long slots = (s1 - 1) / hop - s0 / hop + 1;  // (afs_tree.h plan_hop_slots)
  for (int r = 0; r < rows; ++r)
    for (long q = 0; q < slots; ++q) {
      const long h = s0 / hop + q;
      const long lo = h * hop > s0 ? h * hop : s0, hi = (h + 1) * hop < s1 ? (h + 1) * hop : s1;
      const afs_frame *f = frames + (long)r * F;
      tree::plan_hop_host(f + h, f + h + 1, hop, (int)(lo - h * hop), (int)(hi - h * hop), T.consts.sec,
                          two_mass != 0, out[(long)r * slots + q]);
    }
  return 0;
}

// The interval decisions of K5's hop mode (tree_plan.h plan_hop_decide_iv) against the per-sample
// decisions: for every hop that samples [s0, s1) of frames[rows][F] span, a hop the interval
// evaluation decides must give every one of its samples the same PlanKey as plan_decide on that
// sample.  counts[0]: hops decided, [1]: hops left to the per-sample path, [2]: violations (decided
// hops with a sample whose key differs), [3]: hops whose samples do not all share one key.
extern "C" int emu_plan_iv_check(const afs_frame *frames, int rows, int F, int hop, long s0, long s1, long *counts) {
  for (int q = 0; q < 4; ++q) counts[q] = 0;
  const long slots = (s1 - 1) / hop - s0 / hop + 1;
  for (int r = 0; r < rows; ++r)
    for (long q = 0; q < slots; ++q) {
      const long h = s0 / hop + q;
      const long lo = h * hop > s0 ? h * hop : s0, hi = (h + 1) * hop < s1 ? (h + 1) * hop : s1;
      const afs_frame *fl = frames + (long)r * F + h, *fr = fl + 1;
      const int i0 = (int)(lo - h * hop), i1 = (int)(hi - h * hop);
      tree::PlanKey kiv;
      const bool dec = tree::plan_hop_decide_iv<false>(fl, fr, hop, i0, i1, kiv);
      uint64_t qiv[2], q0[2] = {0, 0};
      tree::plan_key_pack(kiv, qiv);
      bool same = true, viol = false;
      for (int i = i0; i < i1; ++i) {
        const double ratio = (double)i / (double)hop;
        const tree::PlanGeomT<false> g{fl, fr, 1.0 - ratio, ratio};
        tree::PlanKey k;
        double obst[4], po[4];
        tree::plan_decide(g, k, obst, po);
        uint64_t qq[2];
        tree::plan_key_pack(k, qq);
        if (i == i0) { q0[0] = qq[0]; q0[1] = qq[1]; }
        same = same && qq[0] == q0[0] && qq[1] == q0[1];
        viol = viol || (dec && (qq[0] != qiv[0] || qq[1] != qiv[1]));
      }
      counts[dec ? 0 : 1] += 1;
      counts[2] += viol ? 1 : 0;
      counts[3] += same ? 0 : 1;
    }
  return 0;
}

// The words of a hop record at `ratio` (tree_plan.h plan_word_eval, the host form of the
// synthesis kernel's plan_word_fast): out[PLAN_WORDS].
extern "C" void emu_plan_hop_words(const tree::PlanHop *h, double ratio, uint64_t *out) {
  for (int q = 0; q < tree::PLAN_WORDS; ++q) out[q] = tree::plan_word_eval(h->kind[q], h->p[q], ratio);
}
