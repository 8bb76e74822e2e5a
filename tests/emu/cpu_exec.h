// cpu_exec.h -- TEST-ONLY: the host executor of the tree kernel's phase code (tree_emu.cpp,
// pair_emu.cpp): the W lanes of an utterance run one after another; the collectives (DPP pulls,
// ballots, scans) are restated over the lane array.  Included after tree_core.h.
#pragma once
#include <condition_variable>
#include <mutex>
#include <vector>

// Two threads' workgroup barrier (the wave pairs' x.bar(); pair_emu.cpp runs each role on a thread).
struct Barrier2 {
  std::mutex m;
  std::condition_variable cv;
  int count = 0;
  long gen = 0;
  void wait() {
    std::unique_lock<std::mutex> l(m);
    const long g = gen;
    if (++count == 2) {
      count = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(l, [&] { return gen != g; });
    }
  }
};

namespace {

template <int W, bool TONE = false>
struct CpuExec {
  static constexpr bool kGlottisSplit = false;  // (the device's lane split of the glottis masses)
  static constexpr bool kToneOut = TONE;        // the device's tone filter in K6 (emu_tree_set_tone_k6)
  Lane<W> *R;
  Barrier2 *barrier = nullptr;  // (wave pairs, pair_emu.cpp: the two roles' threads meet here)
  int prio = 0;                 // (the device's issue-priority mode: no effect on the host)
  void bar() {
    if (barrier) barrier->wait();
  }
  template <class F> void par(F f) { for (int gl = 0; gl < W; ++gl) f(gl, R[gl]); }
  template <class F> void one(F f) { f(R[0]); }
  const Lane<W> &first() const { return R[0]; }
  template <class F, class G> void par_uniform(F f, G g) { par(f); g(R[0]); }
  template <class F> void lanes(int n, F f) { for (int k = 0; k < n; ++k) f(k, R[k]); }
  void dyn_neighbors() {
    using S = Shape<W>;
    for (int gl = 0; gl < W; ++gl)
      for (int j = 0; j < S::ND; ++j) {
        const int k = j * W + gl, kn = k + 1, kp = k - 1;
        R[gl].anx[j] = kn < S::ND * W ? R[kn % W].acur[kn / W] : 0.0;
        R[gl].apv[j] = kp >= 0 ? R[kp % W].acur[kp / W] : 0.0;
      }
  }
  void sync() {}
  void mark(int) {}
  template <int K> uint64_t rec() { return R[K].planw; }  // lane K holds plan word K
  template <class F> uint64_t ballot(F f) {
    uint64_t m = 0;
    for (int gl = 0; gl < W; ++gl)
      if (f(gl, R[gl])) m |= 1ull << gl;
    return m;
  }
  template <class F> MinIdx min_index(F f) {
    MinIdx b = f(0, R[0]);
    for (int gl = 1; gl < W; ++gl) b = min_idx_combine(b, f(gl, R[gl]));
    return b;
  }
  template <int N, class F, class G> void scan_add(F f, G g) {
    std::vector<U4> out(W);
    U4 acc{{0u, 0u, 0u, 0u}};
    for (int gl = 0; gl < W; ++gl) {
      const U4 v = f(gl, R[gl]);
      for (int i = 0; i < N; ++i) acc.v[i] += v.v[i];
      out[gl] = acc;
    }
    for (int gl = 0; gl < W; ++gl) g(gl, R[gl], out[gl]);
  }
  template <int K, int N, class F, class G> void pull(F f, G g) {
    std::vector<D4> v(W);
    for (int gl = 0; gl < W; ++gl) v[gl] = f(gl, R[gl]);
    for (int gl = 0; gl < W; ++gl) {
      const int src = gl + K;
      D4 o{{0.0, 0.0, 0.0, 0.0}};
      if (src >= 0 && src < W && src / 16 == gl / 16)  // (one 16-lane DPP row on the device)
        for (int i = 0; i < N; ++i) o.v[i] = v[src].v[i];
      g(gl, R[gl], o);
    }
  }
  template <int K, int N, class F, class G> void pull_u(F f, G g) {
    std::vector<U4> v(W);
    for (int gl = 0; gl < W; ++gl) v[gl] = f(gl, R[gl]);
    for (int gl = 0; gl < W; ++gl) {
      const int src = gl + K;
      U4 o{{0u, 0u, 0u, 0u}};
      if (src >= 0 && src < W && src / 16 == gl / 16)
        for (int i = 0; i < N; ++i) o.v[i] = v[src].v[i];
      g(gl, R[gl], o);
    }
  }
  template <int K, int N, class F, class G> void bcast_u(F f, G g) {
    std::vector<U4> v(W);
    for (int gl = 0; gl < W; ++gl) v[gl] = f(gl, R[gl]);
    for (int gl = 0; gl < W; ++gl) {
      U4 o{{0u, 0u, 0u, 0u}};
      for (int i = 0; i < N; ++i) o.v[i] = v[gl / 16 * 16 + K].v[i];
      g(gl, R[gl], o);
    }
  }
  static bool wave_any(bool p) { return p; }  // (one utterance: its lanes agree)
  template <class F> double max_value(F f) {
    double b = f(0, R[0]);
    for (int gl = 1; gl < W; ++gl) b = max_combine(b, f(gl, R[gl]));
    return b;
  }
};

}  // namespace
