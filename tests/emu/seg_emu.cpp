// seg_emu.cpp -- TEST-ONLY host execution of the segment-aligned kernel's phase code.
//
// Runs csrc/seg_core.h's seg_sample_step with the 16 lanes of each phase executed one after
// another (cross-lane values are gathered from every lane before any lane consumes them, as a
// DPP row operation delivers them), so the lane partition, the static condensation and the
// dynamic walks can be checked against the oracle on the CPU.  Never part of the product;
// libafs.so does not contain it.
#include <cstring>
#include <vector>

#include "seg_core.h"

using namespace afs;
using namespace afs::seg;

namespace {

struct SegCpuExec {
  SegLane *R;
  template <class F> void par(F f) { for (int gl = 0; gl < SW; ++gl) f(gl, R[gl]); }
  template <class F, class G> void par_uniform(F f, G g) { par(f); g(R[0]); }
  void sync() {}
  void mark(int) {}
  template <int K> uint64_t rec() { return R[K].planw; }
  template <class F> uint64_t ballot(F f) {
    uint64_t m = 0;
    for (int gl = 0; gl < SW; ++gl)
      if (f(gl, R[gl])) m |= 1ull << gl;
    return m;
  }
  template <class F> uint64_t or64(F f) {
    uint64_t m = 0;
    for (int gl = 0; gl < SW; ++gl) m |= f(gl, R[gl]);
    return m;
  }
  template <int N, class F, class G> void scan_add(F f, G g) {
    std::vector<tree::U4> out(SW);
    tree::U4 acc{{0u, 0u, 0u, 0u}};
    for (int gl = 0; gl < SW; ++gl) {
      const tree::U4 v = f(gl, R[gl]);
      for (int i = 0; i < N; ++i) acc.v[i] += v.v[i];
      out[gl] = acc;
    }
    for (int gl = 0; gl < SW; ++gl) g(gl, R[gl], out[gl]);
  }
  template <int K, int N, class F, class G> void pull(F f, G g) {
    std::vector<tree::D4> v(SW);
    for (int gl = 0; gl < SW; ++gl) v[gl] = f(gl, R[gl]);
    for (int gl = 0; gl < SW; ++gl) {
      const int src = gl + K;
      tree::D4 o{{0.0, 0.0, 0.0, 0.0}};
      if (src >= 0 && src < SW)
        for (int i = 0; i < N; ++i) o.v[i] = v[src].v[i];
      g(gl, R[gl], o);
    }
  }
  template <int K, int N, class F, class G> void bcast(F f, G g) {
    std::vector<tree::D4> v(SW);
    for (int gl = 0; gl < SW; ++gl) v[gl] = f(gl, R[gl]);
    tree::D4 o{{0.0, 0.0, 0.0, 0.0}};
    for (int i = 0; i < N; ++i) o.v[i] = v[K].v[i];
    for (int gl = 0; gl < SW; ++gl) g(gl, R[gl], o);
  }
};

long run(const afs_frame *frames, int F, int hop, unsigned seed, double fs, const afs_options &opt, double *out,
         int64_t *draws) {
  static Tables T;
  static SegTables S;
  build_tables(&T, fs, opt);
  build_seg_tables(T, &S);
  if (!S.ok) return -3;
  std::vector<SegLane> R(SW);
  for (int gl = 0; gl < SW; ++gl) seg_reset_lane(R[gl]);
  std::vector<double> X(SX_STRIDE);
  seg_reset_lds(X.data(), seed);
  seg_init_lds(X.data(), S);
  SegCpuExec ex{R.data()};
  SegHot H{T.consts.h};
  const bool defer = hop >= tree::OUT_DEFER_MIN_HOP;
  const bool two = opt.glottis_model == AFS_GLOTTIS_TWO_MASS;
  long t = 0;
  for (int k = 1; k < F; ++k) {
    for (int gl = 0; gl < SW; ++gl) seg_frame_load(gl, R[gl], X.data(), S.c, frames + k - 1, frames + k);
    const long t0 = t;
    for (int i = 0; i < hop; ++i) {
      const double ratio = (double)i / (double)hop;
      uint64_t w[tree::PLAN_WORDS];
      tree::plan_sample(frames + k - 1, frames + k, ratio, S.uo, two, w);
      for (int gl = 0; gl < SW; ++gl) R[gl].planw = w[gl % tree::PLAN_WORDS];
      if (two) seg_sample_step<AFS_GLOTTIS_TWO_MASS>(ex, X.data(), T.uni, H, S.c, ratio, defer);
      else seg_sample_step<AFS_GLOTTIS_TRIANGULAR>(ex, X.data(), T.uni, H, S.c, ratio, defer);
      out[t] = R[0].sample;
      ++t;
    }
    if (defer) seg_output_filter_run(X.data(), H, out + t0, hop);
  }
  if (draws) *draws = (int64_t) * (const uint64_t *)(X.data() + SX_NDRAW);
  return t;
}

}  // namespace

// options as tests/emu/tree_emu.cpp: turbulence, soft walls, noise, skin radiation, fossa,
// inner length corrections, transvelar coupling, glottis loss, glottis model (ints) and the
// flow-separation area ratio; iopt == NULL: TdsModel's defaults.
extern "C" long emu_seg_utterance(const afs_frame *frames, int F, int hop, unsigned seed, double fs, const int *iopt,
                                  double ratio, double *out, int64_t *draws) {
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
  return run(frames, F, hop, seed, fs, opt, out, draws);
}

extern "C" int emu_seg_tables_ok(double fs) {
  static Tables T;
  static SegTables S;
  build_tables(&T, fs, afs::default_options());
  build_seg_tables(T, &S);
  return S.ok;
}

// The noise-source plan records (tree_plan.h plan_sample, as K5 evaluates them) of samples
// [s0, s1) of frames[rows][F] at this hop: out[rows][s1 - s0][PLAN_WORDS].  seg_layout: the X_UN
// offsets of the seg kernel's LDS layout instead of the tree kernel's.
extern "C" int emu_plan_records(const afs_frame *frames, int rows, int F, int hop, long s0, long s1, double fs,
                                int two_mass, int seg_layout, uint64_t *out) {
  static Tables T;
  static SegTables S;
  afs_options opt = afs::default_options();
  opt.glottis_model = two_mass ? AFS_GLOTTIS_TWO_MASS : AFS_GLOTTIS_TRIANGULAR;
  build_tables(&T, fs, opt);
  const SecRec *uo = T.consts.sec;
  if (seg_layout) {
    build_seg_tables(T, &S);
    if (!S.ok) return -3;
    uo = S.uo;
  }
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
