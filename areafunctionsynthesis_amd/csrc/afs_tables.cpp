// afs_tables.cpp -- host-side evaluation of everything static in the tube network.
//
// All values are computed with the reference's formulas and operand order in plain
// IEEE double (no FMA contraction: this file is built with -ffp-contract=off), so the
// constants the kernels read are bit-identical to what the reference recomputes each
// sample for the same sections.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <initializer_list>
#include <vector>

#include "afs_model.h"
#include "tree_core.h"

namespace afs {

namespace {

const double NOSE_AREA[19] = {1.63, 2.07, 2.72, 3.59, 4.24, 3.26, 3.04, 3.04, 2.72, 2.5,
                              2.39, 2.39, 1.85, 0.76, 1.41, 1.74, 1.30, 1.74, 0.76};  // Tube.cpp:155-157
const double SINUS_VOLUME[4] = {11.3, 6.8, 33.0, 6.2};                                 // Tube.cpp:159
const double NECK_LENGTH[4] = {0.3, 0.3, 0.45, 1.0};                                   // Tube.cpp:160
const double NECK_AREA[4] = {0.185, 0.185, 0.145, 0.11};                               // Tube.cpp:161
const int SINUS_COUPLING[4] = {8, 9, 11, 12};                                          // Tube.cpp:35-38

// Static geometry and wall data (Tube.cpp:79-314).
void static_geometry(Tables *t) {
  for (int i = 0; i < NS; ++i) {
    t->Mw[i] = 2.1; t->Bw[i] = 800.0; t->Kw[i] = 84500.0;
    t->area[i] = 0.0; t->len[i] = 0.0; t->vol[i] = 0.0;
  }
  for (int i = 0; i <= S_LAST_TRACHEA; ++i) {
    t->area[i] = (i == 0) ? 4.0 : (i == 1) ? 3.0 : 2.5;
    t->len[i] = 23.0 / (double)23;
    t->vol[i] = t->area[i] * t->len[i];
    t->Mw[i] = 0.25; t->Bw[i] = 1000.0;
  }
  const double lf = 11.4 / 11.4;
  for (int i = 0; i < 19; ++i) {
    int k = S_NOSE0 + i;
    t->area[k] = NOSE_AREA[i];
    t->len[k] = lf * 0.6;
    t->vol[k] = t->area[k] * t->len[k];
  }
  for (int i = 0; i < 4; ++i) {
    int k = S_SINUS0 + i;
    t->area[k] = NECK_AREA[i]; t->len[k] = NECK_LENGTH[i]; t->vol[k] = SINUS_VOLUME[i];
    t->Mw[k] = 0.0; t->Bw[k] = 6500.0;
  }
  const double amax = 2.0 * 2.0 / 3.0, sl = 3.0 / (double)5;
  for (int i = 0; i < 5; ++i) {
    int k = S_FOSSA0 + i;
    t->area[k] = amax * (1.0 - (i + 0.5) / (double)5);
    t->len[k] = sl;
    t->vol[k] = t->area[k] * t->len[k];
  }
  t->nose4_area = t->area[S_NOSE0 + 4];
}

// prepareTimeStep's per-section terms for sections whose geometry never changes
// (TdsModel.cpp:741-832 and :988-1008 for E).
void static_network(Tables *t) {
  const double dt = t->dt;
  for (int i = 0; i < NS; ++i) {
    t->L[i] = t->C[i] = t->R[i] = t->alpha[i] = t->wc1[i] = t->wc2[i] = t->Lw[i] = t->E[i] = 0.0;
    if (!is_static_section(i)) continue;
    double area = t->area[i], len = t->len[i], vol = t->vol[i];
    double circ = 2.0 * std::sqrt(area * PI);
    if (i >= S_SINUS0 && i <= S_LAST_SINUS) {
      t->L[i] = RHO * (len / area);
      t->C[i] = vol / (RHO * CSND * CSND);
      t->R[i] = (8.0 * MU * PI * len) / (area * area);
    } else {
      double a = std::sqrt(area / PI), b = a;
      const double rmin = 1.6;
      if (a < rmin) { a = rmin; b = area / (PI * a); }
      t->L[i] = (RHO * 0.5 * len) / area;
      t->C[i] = vol / (RHO * CSND * CSND);
      t->R[i] = ((2.0 * MU * len) * (a * a + b * b)) / (PI * a * a * a * b * b * b);
    }
    if (t->opt.soft_walls) {
      double surf;
      if (i >= S_SINUS0 && i <= S_LAST_SINUS)
        surf = 4.0 * PI * std::pow((3.0 * vol) / (4.0 * PI), 2.0 / 3.0);
      else
        surf = circ * len;
      if (surf < AMIN) surf = AMIN;
      double Rw = t->Bw[i] / surf, Lw = t->Mw[i] / surf, Cw = surf / t->Kw[i];
      t->alpha[i] = 1.0 / (Lw / (dt * dt * TH * TH) + Rw / (dt * TH) + 1.0 / Cw);
      t->wc1[i] = Lw / (dt * dt * TH * TH) + Rw / (dt * TH);
      t->wc2[i] = Lw * (TH1 / TH + 1.0) / (dt * TH) + Rw * (TH1 / TH);
      t->Lw[i] = Lw;
    }
    t->E[i] = dt * TH / (t->C[i] + t->alpha[i]);
  }
}

void topology(Tables *t) {
  for (int i = 0; i < NS; ++i) { t->src[i] = (int16_t)(i - 1); t->tgt[i] = (int16_t)i; }
  t->src[0] = -1;
  t->src[S_NOSE0] = S_LAST_PHARYNX;
  t->src[S_FOSSA0] = S_PHARYNX0 + 3;
  for (int i = 0; i < 4; ++i) t->src[S_SINUS0 + i] = (int16_t)(S_NOSE0 + SINUS_COUPLING[i]);
  t->src[93] = t->src[94] = S_LAST_MOUTH;
  t->src[95] = t->src[96] = S_LAST_NOSE;
  t->tgt[93] = t->tgt[94] = t->tgt[95] = t->tgt[96] = -1;
  for (int s = 0; s < NS; ++s) t->cin[s] = t->cout0[s] = t->cout1[s] = -1;
  for (int c = 0; c < NC; ++c) {
    if (t->src[c] != -1) {
      int s = t->src[c];
      if (t->cout0[s] == -1) t->cout0[s] = (int16_t)c; else t->cout1[s] = (int16_t)c;
    }
    if (t->tgt[c] != -1) t->cin[t->tgt[c]] = (int16_t)c;
  }
  // Matrix pattern and the envelope (TdsModel.cpp:218-292).
  static unsigned char nz[NC][NC];
  std::memset(nz, 0, sizeof nz);
  int off = 0;
  for (int c = 0; c < NC; ++c) {
    const int sides[2] = {t->src[c], t->tgt[c]};
    for (int s : sides) {
      if (s == -1) continue;
      if (t->cin[s] != -1) nz[c][t->cin[s]] = 1;
      if (t->cout0[s] != -1) nz[c][t->cout0[s]] = 1;
      if (t->cout1[s] != -1) nz[c][t->cout1[s]] = 1;
    }
    t->row_n[c] = 0;
    for (int j = 0; j < NC; ++j)
      if (nz[c][j] && j != c && t->row_n[c] < 16) t->row[c][t->row_n[c]++] = (int16_t)j;
    int first = c;
    for (int j = 0; j < c; ++j)
      if (nz[c][j]) { first = j; break; }
    for (int j = first; j < c; ++j) nz[c][j] = 1;
    t->env_start[c] = (int16_t)first;
    t->env_n[c] = (int16_t)(c - first);
    t->env_off[c] = (int16_t)off;
    off += c - first;
  }
  t->env_total = off;
  for (int j = 0; j < NC; ++j) {
    int n = 0;
    for (int i = j + 1; i < NC; ++i)
      if (nz[i][j]) t->col[j][n++] = (int16_t)i;
    t->col_n[j] = (int16_t)n;
  }
}

// Edge numbering of the current graph (afs_model.h); the arm solver's records address the
// edges' LDS slots by these ids.
bool edge_numbering(Tables *t) {
  int e = 0;
  for (int s = 0; s < NS; ++s) {
    t->edge[s][0] = t->edge[s][1] = t->edge[s][2] = -1;
    if (t->cout0[s] != -1) t->edge[s][0] = (int16_t)e++;
    if (t->cout1[s] != -1) {
      t->edge[s][1] = (int16_t)e++;
      t->edge[s][2] = (int16_t)e++;
    }
  }
  t->n_edges = e;
  return e == TREE_NE;
}

// The arm solver's lane records (afs_model.h ArmRec, tree_core.h solve_arms).  The partition
// (tools/arm_solver_study.py checks the elimination on random SPD systems): per lane the
// segment from the far end to its boundary, then the fold leaves.  The builder checks that
// the roles it assigns use every edge of the current graph exactly once (chain edges, anchor
// edges between consecutive lanes of an arm, fold edges, the fossa's two edges, the three
// arm-to-junction edges, the triangle) and every current exactly once; with that, the
// elimination the kernel performs is the exact LDL^T of the system.
bool arm_records(Tables *t) {
  static const int SEG[TREE_CHAINS][ARM_P] = {
      // arm A (far end 0), walked upward
      {0, 1, 2, 3, 4, 5, 6, -1}, {7, 8, 9, 10, 11, 12, 13, -1}, {14, 15, 16, 17, 18, 19, 20, -1},
      {21, 22, 23, 24, 25, 26, 27, 28}, {29, -1}, {30, 31, 32, 33, 34, -1}, {35, 36, 37, 38, 39, -1},
      // arm B (far end: the radiation pair), walked downward
      {93, 64, 63, 62, 61, 60, -1}, {59, 58, 57, 56, 55, 54, -1}, {53, 52, 51, 50, 49, 48, -1},
      {47, 46, 45, 44, 43, 42, -1},
      // arm C (far end: the nostril pair)
      {96, 83, 82, 81, 80, 79, -1}, {78, 77, 76, 75, 74, 73, -1}, {72, 71, 70, 69, 68, 67, 66, -1},
      // fossa (84 is its boundary), junction (no segment)
      {88, 87, 86, 85, 84, -1}, {-1}};
  static const int ARM_OF[TREE_CHAINS] = {0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, -1, -1};
  static const int LEAF[TREE_CHAINS][ARM_FOLDS] = {
      {-1, -1, -1, -1}, {-1, -1, -1, -1}, {-1, -1, -1, -1}, {-1, -1, -1, -1}, {-1, -1, -1, -1},
      {-1, -1, -1, -1}, {-1, -1, -1, -1}, {94, -1, -1, -1}, {-1, -1, -1, -1}, {-1, -1, -1, -1},
      {-1, -1, -1, -1}, {95, -1, -1, -1}, {92, 91, 90, 89}, {-1, -1, -1, -1}, {-1, -1, -1, -1},
      {-1, -1, -1, -1}};
  static const int JN[3] = {40, 41, 65}, JEND[3] = {39, 42, 66};
  static int16_t eid[NC][NC];
  for (int i = 0; i < NC; ++i)
    for (int j = 0; j < NC; ++j) eid[i][j] = -1;
  for (int s = 0; s < NS; ++s) {
    const int m[3] = {t->cin[s], t->cout0[s], t->cout1[s]};
    const int pk[3][3] = {{-1, 0, 1}, {0, -1, 2}, {1, 2, -1}};
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b)
        if (a != b && m[a] >= 0 && m[b] >= 0) eid[m[a]][m[b]] = t->edge[s][pk[a][b]];
  }
  using namespace tree;
  auto off = [](int slot) { return (uint16_t)(slot * 8); };
  const uint16_t ONE = off(X_DIAG + NC + 1), ZE = off(X_OFF + EDGE_ZERO), USINK = off(X_U + U_SINK);
  std::vector<int> edge_uses(TREE_NE, 0), node_uses(NC, 0);
  bool ok = true;
  auto use_edge = [&](int a, int b) -> uint16_t {
    if (a < 0 || b < 0 || a >= NC || b >= NC || eid[a][b] < 0 || eid[a][b] >= TREE_NE) { ok = false; return ZE; }
    edge_uses[eid[a][b]]++;
    return off(X_OFF + eid[a][b]);
  };
  int bound[TREE_CHAINS];
  Consts &c = t->consts;
  for (int k = 0; k < TREE_CHAINS; ++k) {
    int n = 0;
    while (n < ARM_P && SEG[k][n] >= 0) ++n;
    ArmRec &r = c.arm[k];
    std::memset(&r, 0, sizeof r);
    const int start = ARM_P - n;
    int pos[ARM_P];
    for (int p = 0; p < ARM_P; ++p) pos[p] = p >= start ? SEG[k][p - start] : -1;
    bound[k] = n ? pos[ARM_P - 1] : -1;
    r.start = (uint8_t)start;
    if (start > ARM_START_MAX && start < ARM_P - 1) ok = false;  // (the walk's anchor-edge positions)
    for (int p = 0; p < ARM_P; ++p) {
      if (pos[p] >= 0) node_uses[pos[p]]++;
      r.d[p] = pos[p] >= 0 ? off(X_DIAG + pos[p]) : ONE;
      r.u[p] = pos[p] >= 0 ? off(X_U + pos[p]) : USINK;
    }
    for (int p = 0; p + 1 < ARM_P; ++p) r.e[p] = (pos[p] >= 0) ? use_edge(pos[p], pos[p + 1]) : ZE;
    // anchor: the previous lane of the same arm
    const bool anchored = ARM_OF[k] >= 0 && k > 0 && ARM_OF[k - 1] == ARM_OF[k];
    r.ea = (anchored && n) ? use_edge(bound[k - 1], pos[start]) : ZE;
    int idx = 0;
    for (int j = k - 1; j >= 0 && ARM_OF[j] == ARM_OF[k] && ARM_OF[k] >= 0; --j) ++idx;
    r.idx = (uint8_t)(ARM_OF[k] >= 0 ? idx : 0xff);
    const bool last = ARM_OF[k] >= 0 && (k + 1 == TREE_CHAINS || ARM_OF[k + 1] != ARM_OF[k]);
    r.flags = (uint8_t)((ARM_OF[k] >= 0 ? ARM_IN : 0) | (last ? ARM_END : 0));
    r.ej = ZE;
    if (last) r.ej = use_edge(JEND[ARM_OF[k]], JN[ARM_OF[k]]);
    if (last && bound[k] != JEND[ARM_OF[k]]) ok = false;
    for (int f = 0; f < ARM_FOLDS; ++f) {
      const int leaf = LEAF[k][f], p = arm_fold_pos(f);
      r.ld[f] = leaf >= 0 ? off(X_DIAG + leaf) : ONE;
      r.lu[f] = leaf >= 0 ? off(X_U + leaf) : USINK;
      r.le0[f] = leaf >= 0 ? use_edge(leaf, pos[p]) : ZE;
      r.le1[f] = leaf >= 0 ? use_edge(leaf, pos[p + 1]) : ZE;
      if (leaf >= 0) node_uses[leaf]++;
    }
    r.fx0 = r.fx1 = ZE;
  }
  // roles fixed in the kernel
  if (bound[ARM_L28] != 28 || bound[ARM_L28 + 1] != 29 || bound[ARM_FOSSA] != 84 || bound[ARM_JUNCTION] != -1 ||
      bound[ARM_END_A] != 39 || bound[ARM_END_B] != 42 || bound[ARM_END_C] != 66)
    ok = false;
  c.arm[ARM_FOSSA].fx0 = use_edge(84, 28);
  c.arm[ARM_FOSSA].fx1 = use_edge(84, 29);
  ArmJunction &j = c.armj;
  std::memset(&j, 0, sizeof j);
  for (int q = 0; q < 3; ++q) {
    j.d[q] = off(X_DIAG + JN[q]);
    j.u[q] = off(X_U + JN[q]);
    node_uses[JN[q]]++;
  }
  j.e[0] = use_edge(40, 41);
  j.e[1] = use_edge(40, 65);
  j.e[2] = use_edge(41, 65);
  for (int e = 0; e < TREE_NE; ++e) ok = ok && edge_uses[e] == 1;
  for (int i = 0; i < NC; ++i) ok = ok && node_uses[i] == 1;
  return ok;
}

// LDS slots of the edges (X_OFF), chosen for the LDS banks.  The kernel reads and writes the edges
// through its records, 16 lanes of an utterance per instruction: the row phase the edges of the
// sections of one slot, the arm solver those of one position of every lane's segment.  Two
// utterances share a 32-lane bank group (their blocks X_STRIDE = 16 mod 32 doubles apart), so the
// lanes of one instruction are conflict-free when their edges' slots differ modulo 16 doubles
// (MI355X_MICROARCH.md §LDS).  Numbered in graph order, lanes k and k + 5 of an arm position met
// on one bank (tools/lds_banks.cpp); here every edge gets a residue modulo 16 that minimises the
// clashes within the access groups (greedy, then single moves and swaps until none helps), and
// the residue classes are laid out over the slots.  The edges' values are the same; only where
// they sit changes.
void bank_edge_slots(Consts &c) {
  using namespace tree;
  constexpr int R = 16;
  auto id_of = [](uint16_t v) -> int {  // the zero and sink edges keep their slots TREE_NE, TREE_NE + 1
    const int slot = (int)(v / 8) - X_OFF;
    return (slot >= 0 && slot < TREE_NE + 2) ? slot : -1;
  };
  std::vector<std::vector<int>> groups;
  auto add = [&](const std::vector<int> &g) {
    std::vector<int> u;
    for (int e : g)
      if (e >= 0 && std::find(u.begin(), u.end(), e) == u.end()) u.push_back(e);
    if (u.size() > 1) groups.push_back(u);
  };
  constexpr int W = 16;
  for (int j = 0; j < Shape<W>::NSL; ++j) {
    std::vector<int> g0, g1, g2;
    for (int gl = 0; gl < W; ++gl) {
      const int s0 = slot_section<W>(j, gl);
      const SecRec &q = c.sec[s0 < 0 ? NS : s0];
      g0.push_back(id_of(q.x_e0));
      g1.push_back(id_of(q.x_e1));
      g2.push_back(id_of(q.x_e2));
    }
    add(g0), add(g1), add(g2);
  }
  for (int p = 0; p + 1 < ARM_P; ++p) {
    std::vector<int> g;
    for (int k = 0; k < TREE_CHAINS; ++k) g.push_back(id_of(c.arm[k].e[p]));
    add(g);
  }
  {
    std::vector<int> ga, gj, gx;
    for (int k = 0; k < TREE_CHAINS; ++k) {
      ga.push_back(id_of(c.arm[k].ea));
      gj.push_back(id_of(c.arm[k].ej));
      gx.push_back(id_of(c.arm[k].fx0));
      gx.push_back(id_of(c.arm[k].fx1));
    }
    add(ga), add(gj), add(gx);
  }
  for (int f = 0; f < ARM_FOLDS; ++f) {
    std::vector<int> g0, g1;
    for (int k = 0; k < TREE_CHAINS; ++k) {
      g0.push_back(id_of(c.arm[k].le0[f]));
      g1.push_back(id_of(c.arm[k].le1[f]));
    }
    add(g0), add(g1);
  }
  int cap[R] = {};
  for (int sl = 0; sl < TREE_NE; ++sl) cap[(X_OFF + sl) % R]++;
  std::vector<int> res(TREE_NE + 2, -1), used(R, 0);
  res[TREE_NE] = (X_OFF + TREE_NE) % R;  // (fixed)
  res[TREE_NE + 1] = (X_OFF + TREE_NE + 1) % R;
  std::vector<std::vector<int>> of(TREE_NE + 2);  // groups of an edge
  for (int gi = 0; gi < (int)groups.size(); ++gi)
    for (int e : groups[gi]) of[e].push_back(gi);
  auto clash = [&](int e, int r) {  // edges of e's groups on residue r
    int n = 0;
    for (int gi : of[e])
      for (int f : groups[gi]) n += f != e && res[f] == r;
    return n;
  };
  // greedy, the edges in most groups first
  std::vector<int> order(TREE_NE);
  for (int e = 0; e < TREE_NE; ++e) order[e] = e;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return of[a].size() > of[b].size(); });
  for (int e : order) {
    int best = -1, bc = 1 << 30;
    for (int r = 0; r < R; ++r)
      if (used[r] < cap[r]) {
        const int cc = clash(e, r);
        if (cc < bc) bc = cc, best = r;
      }
    res[e] = best;
    used[best]++;
  }
  for (bool better = true; better;) {
    better = false;
    for (int e = 0; e < TREE_NE; ++e) {
      const int r0 = res[e], c0 = clash(e, r0);
      if (c0 == 0) continue;
      for (int r = 0; r < R && !better; ++r) {
        if (r == r0) continue;
        if (used[r] < cap[r]) {  // move
          if (clash(e, r) < c0) {
            res[e] = r, used[r]++, used[r0]--, better = true;
          }
          continue;
        }
        for (int f = 0; f < TREE_NE && !better; ++f) {  // swap with an edge on r
          if (res[f] != r) continue;
          const int before = c0 + clash(f, r);
          res[e] = r, res[f] = r0;
          if (clash(e, r) + clash(f, r0) < before) better = true;
          else res[e] = r0, res[f] = r;
        }
      }
    }
  }
  // residue classes over the slots, in edge order within a class
  std::vector<int> slot(TREE_NE, -1), next(R, 0);
  std::vector<std::vector<int>> slots_of(R);
  for (int sl = 0; sl < TREE_NE; ++sl) slots_of[(X_OFF + sl) % R].push_back(sl);
  for (int e = 0; e < TREE_NE; ++e) slot[e] = slots_of[res[e]][next[res[e]]++];
  auto remap = [&](uint16_t &v) {
    const int e = id_of(v);
    if (e >= 0 && e < TREE_NE) v = (uint16_t)((X_OFF + slot[e]) * 8);
  };
  for (int s = 0; s <= NS; ++s) remap(c.sec[s].x_e0), remap(c.sec[s].x_e1), remap(c.sec[s].x_e2);
  for (int k = 0; k < TREE_CHAINS; ++k) {
    ArmRec &r = c.arm[k];
    for (int p = 0; p + 1 < ARM_P; ++p) remap(r.e[p]);
    remap(r.ea), remap(r.ej), remap(r.fx0), remap(r.fx1);
    for (int f = 0; f < ARM_FOLDS; ++f) remap(r.le0[f]), remap(r.le1[f]);
  }
  for (int q = 0; q < 3; ++q) remap(c.armj.e[q]);
}

}  // namespace

// IirFilter::createChebyshev, IirFilter.cpp:286-432 (0.5 % ripple).
int chebyshev(double ratio, bool hp, int poles, double *aout, double *bout) {
  double a[33], b[33], ta[33], tb[33];
  if (poles & 1) poles++;
  if (poles > 32) poles = 32;
  for (int i = 0; i <= 32; ++i) a[i] = b[i] = 0.0;
  a[2] = 1.0;
  b[2] = 1.0;
  for (int p = 1; p <= poles / 2; ++p) {
    double re = -std::cos(PI / (2.0 * poles) + (PI * (p - 1)) / (double)poles);
    double im = std::sin(PI / (2.0 * poles) + (PI * (p - 1)) / (double)poles);
    const double tmp = 100.0 / (100.0 - 0.5);
    const double es = std::sqrt(tmp * tmp - 1.0);
    const double vx = (1.0 / (double)poles) * std::log((1.0 / es) + std::sqrt((1.0 / (es * es)) + 1));
    double kx = (1.0 / (double)poles) * std::log((1.0 / es) + std::sqrt((1.0 / (es * es)) - 1));
    kx = 0.5 * (std::exp(kx) + std::exp(-kx));
    re = re * (0.5 * (std::exp(vx) - std::exp(-vx))) / kx;
    im = im * (0.5 * (std::exp(vx) + std::exp(-vx))) / kx;
    const double t = 2.0 * std::tan(0.5);
    const double w = 2.0 * PI * ratio;
    const double m = re * re + im * im;
    double d = 4.0 - 4.0 * re * t + m * t * t;
    const double x0 = (t * t) / d, x1 = (2.0 * t * t) / d, x2 = (t * t) / d;
    const double y1 = (8.0 - 2.0 * m * t * t) / d;
    const double y2 = (-4.0 - 4.0 * re * t - m * t * t) / d;
    const double k = hp ? -std::cos(0.5 * w + 0.5) / std::cos(0.5 * w - 0.5)
                        : std::sin(0.5 - 0.5 * w) / std::sin(0.5 + 0.5 * w);
    d = 1.0 + y1 * k - y2 * k * k;
    const double a0 = (x0 - x1 * k + x2 * k * k) / d;
    double a1 = (-2.0 * x0 * k + x1 + x1 * k * k - 2.0 * x2 * k) / d;
    const double a2 = (x0 * k * k - x1 * k + x2) / d;
    double b1 = (2.0 * k + y1 + y1 * k * k - 2.0 * y2 * k) / d;
    const double b2 = (-(k * k) - y1 * k + y2) / d;
    if (hp) { a1 = -a1; b1 = -b1; }
    std::memcpy(ta, a, sizeof ta);
    std::memcpy(tb, b, sizeof tb);
    for (int i = 2; i <= 32; ++i) {
      a[i] = a0 * ta[i] + a1 * ta[i - 1] + a2 * ta[i - 2];
      b[i] = tb[i] - b1 * tb[i - 1] - b2 * tb[i - 2];
    }
  }
  b[2] = 0.0;
  for (int i = 0; i <= 30; ++i) { a[i] = a[i + 2]; b[i] = -b[i + 2]; }
  double sa = 0.0, sb = 0.0;
  for (int i = 0; i <= 30; ++i) {
    if (!hp || (i & 1) == 0) { sa += a[i]; sb += b[i]; }
    else { sa -= a[i]; sb -= b[i]; }
  }
  const double gain = sa / (1.0 - sb);
  for (int i = 0; i <= 30; ++i) a[i] /= gain;
  for (int i = 0; i <= poles; ++i) { aout[i] = a[i]; bout[i] = b[i]; }
  return poles;
}

void build_tables(Tables *t, double fs_hz, const afs_options &opt) {
  std::memset(t, 0, sizeof *t);
  t->opt = opt;
  t->fs = fs_hz;
  t->dt = 1.0 / fs_hz;
  t->dtTH = t->dt * TH;
  t->dtTH1 = t->dt * TH1;
  t->th1_th = TH1 / TH;
  t->inv_dtTH = 1.0 / (t->dt * TH);
  t->noise_amp_F = 1.0 - std::exp(-2.0 * PI * 40.0 * t->dt);
  t->noise_lp_c = std::exp(-2.0 * PI * 500.0 * t->dt);
  t->noise_x_2000 = std::exp(-2.0 * PI * (2000.0 * t->dt));
  t->sqrt12 = std::sqrt(12.0);
  t->rrad_num = 128 * RHO * CSND;
  t->lrad_num = 8.0 * RHO;
  static const double TA[5] = {5.027640021717718e-007, -7.995535578908732e-007, 2.967895557191014e-007, 0.0, 0.0};
  static const double TB[5] = {0.0, 3.986308869708467, -5.959669638387298, 3.960408461107104, -0.987047716233603};
  for (int i = 0; i < 5; ++i) { t->tone_a[i] = TA[i]; t->tone_b[i] = TB[i]; }
  chebyshev(7000.0 / fs_hz, false, 8, t->out_a, t->out_b);
  chebyshev(50.0 / fs_hz, false, 4, t->tglot_a, t->tglot_b);
  static const double VA2[5] = {6.589309727087047e-004, -0.001972281980771, 0.001968000742164,
                                -6.546497341015677e-004, 0.0};
  for (int i = 0; i < 5; ++i) t->tvel2_a[i] = VA2[i];
  static_geometry(t);
  static_network(t);
  t->fossa_R0 = 8.0 * MU * t->len[S_FOSSA0] * PI / (AMIN * AMIN);
  topology(t);
  t->n_rounds = (edge_numbering(t) && arm_records(t)) ? ARM_MAXLEN - 1 : -1;
  // packed copy for the cooperative kernel
  Consts &c = t->consts;
  Hot &h = c.h;
  h.fs = t->fs; h.dt = t->dt; h.dtTH1 = t->dtTH1; h.noise_amp_F = t->noise_amp_F; h.noise_lp_c = t->noise_lp_c;
  h.noise_x_2000 = t->noise_x_2000; h.sqrt12 = t->sqrt12; h.nose4_area = t->nose4_area; h.fossa_R0 = t->fossa_R0;
  h.rrad_num = t->rrad_num; h.lrad_num = t->lrad_num;
  for (int i = 0; i < 5; ++i) { h.tone_a[i] = t->tone_a[i]; h.tone_b[i] = t->tone_b[i]; }
  for (int i = 0; i < 9; ++i) { h.out_a[i] = t->out_a[i]; h.out_b[i] = t->out_b[i]; }
  for (int i = 0; i < 5; ++i) { h.tglot_a[i] = t->tglot_a[i]; h.tglot_b[i] = t->tglot_b[i]; h.tvel2_a[i] = t->tvel2_a[i]; }
  h.len_nose0 = t->len[S_NOSE0]; h.Bw_ph0 = t->Bw[S_PHARYNX0]; h.Mw_ph0 = t->Mw[S_PHARYNX0];
  h.Kw_ph0 = t->Kw[S_PHARYNX0]; h.area_last_trachea = t->area[S_LAST_TRACHEA]; h.area_last_nose = t->area[S_LAST_NOSE];
  // the nostrils' radiation elements, as the row phase evaluates them for a static area
  // (tree_core.h radiation_rl; the device's division is within an ulp of this one)
  h.rrad_nose = t->rrad_num / (9.0 * PI * PI * h.area_last_nose);
  h.lrad_nose = t->lrad_num / (3.0 * PI * std::sqrt(h.area_last_nose * PI));
  h.inv_dtTH = 1.0 / (t->dt * TH);
  h.inv_dt2TH2 = 1.0 / (t->dt * t->dt * TH * TH);
  h.Tt = 1.0 / t->fs;
  h.inv_dt = 1.0 / t->dt;
  h.g_smk0 = std::sqrt(G_MASS0 * G_K0);
  h.g_smk1 = std::sqrt(G_MASS1 * G_K1);
  {
    const double gm[2][8] = {{G_MASS0, G_K0, G_KC0, G_DAMP0, h.g_smk0, G_INLET, G_REST_THICK0, 0.0},
                             {G_MASS1, G_K1, G_KC1, G_DAMP1, h.g_smk1, G_OUTLET, G_REST_THICK1, 0.0}};
    for (int i = 0; i < 2; ++i)
      for (int k = 0; k < 8; ++k) h.gmass[i][k] = gm[i][k];
    for (int k = 0; k < 16; ++k) h.gmass_pad[k] = 0.0;
  }
  {
    const double Mw = h.Mw_ph0, Bw = h.Bw_ph0, Kw = h.Kw_ph0;
    const double idt = 1.0 / (t->dt * TH), idt2 = 1.0 / (t->dt * t->dt * TH * TH), th = TH1 / TH;
    const double K = Mw * idt2 + Bw * idt + Kw;
    h.wall_invK = 1.0 / K;
    h.wall_k1 = (Mw * idt2 + Bw * idt) / K;
    h.wall_k2 = (Mw * (th + 1.0) * idt + Bw * th) / K;
    h.wall_k3 = Mw * th / K;
    h.rrad_c = t->rrad_num / (9.0 * PI * PI);
    h.lrad_c = t->lrad_num / (3.0 * PI);
  }
  // step records: LDS byte offsets of the tree kernel's utterance block (tree_core.h)
  using namespace tree;
  // X_UR slots: both outputs of every bifurcation (their partner reads d/dt of the flow)
  std::memset(c.ur_slot, -1, sizeof c.ur_slot);
  int nur = 0;
  for (int s = 0; s < NS; ++s)
    if (t->cout0[s] >= 0 && t->cout1[s] >= 0) {
      if (nur + 2 > NUR) { t->n_rounds = -1; break; }
      c.ur_slot[t->cout0[s]] = (int8_t)nur++;
      c.ur_slot[t->cout1[s]] = (int8_t)nur++;
    }
  // X_UN slots: outputs of the sections a constriction can narrow (24..64) and radiation
  std::memset(c.un_slot, -1, sizeof c.un_slot);
  int nun = 0;
  auto add_un = [&](int i) {
    if (i < 0 || c.un_slot[i] >= 0) return;
    if (nun >= NUN) { t->n_rounds = -1; return; }
    c.un_slot[i] = (int8_t)nun++;
  };
  for (int s = S_GLOT_UP; s <= S_LAST_MOUTH; ++s) { add_un(t->cout0[s]); add_un(t->cout1[s]); }
  add_un(t->cout0[S_LAST_NOSE]);
  add_un(t->cout1[S_LAST_NOSE]);
  t->uni.opt = t->opt;
  for (int s = 0; s < NS; ++s) {
    Topo &q = c.topo[s];
    q.src = (int8_t)t->src[s];
    q.br = -1;
    q.urbr = -1;
    const int a = t->src[s];
    if (a >= 0) {
      const int br = (t->cout0[a] == s) ? t->cout1[a] : t->cout0[a];
      q.br = (int8_t)br;
      if (br >= 0) q.urbr = c.ur_slot[br];
    }
    q.out0 = (int8_t)t->cout0[s];
    q.out1 = (int8_t)t->cout1[s];
    q.e0 = (int8_t)t->edge[s][0];
    q.e1 = (int8_t)t->edge[s][1];
    q.e2 = (int8_t)t->edge[s][2];
  }
  // per-section records of the row and update phases (afs_model.h SecRec)
  const int16_t zero = (int16_t)(X_U + U_ZERO), sink = (int16_t)(X_U + U_SINK);
  auto dyn = [](int s) { return s >= tree::DYN0 && s < tree::DYN0 + tree::NDYNS; };
  for (int s = 0; s <= NS; ++s) {
    SecRec &q = c.sec[s];
    std::memset(&q, 0, sizeof q);
    const bool real = s < NS;
    const int a = real ? t->src[s] : -1;
    int br = -1;
    if (a >= 0) br = (t->cout0[a] == s) ? t->cout1[a] : t->cout0[a];
    const bool da = a >= 0 && dyn(a), sa = a >= 0 && !dyn(a);
    // (a static source or none: entry NDYP - 1 of the dynamic arrays, which no slot writes -- absent
    // slots store into entry NDYNS -- so it stays 0.0 from the reset; the row phase reads L, R1 and
    // E of the source at fixed distances from x_la, tree_core.h phase_rows)
    static_assert(tree::NDYP - 1 > tree::NDYNS, "a dynamic-array entry that no slot writes");
    const int ad = da ? a - tree::DYN0 : tree::NDYP - 1;
    q.x_la = (int16_t)(X_L + ad);
    q.x_ra = (int16_t)(X_R1 + ad);
    q.x_ea = (int16_t)(X_E + ad);
    q.c_la = sa ? t->L[a] : 0.0;
    q.c_ra = sa ? t->R[a] : 0.0;
    q.c_ea = sa ? t->E[a] : 0.0;
    q.x_da = a >= 0 ? (int16_t)(X_D + a) : zero;
    q.x_ub = br >= 0 ? (int16_t)(X_U + br) : zero;
    q.x_urb = br >= 0 && c.ur_slot[br] >= 0 ? (int16_t)(X_UR + c.ur_slot[br]) : zero;
    q.x_sx = (s >= S_PHARYNX0 && s <= S_LAST_MOUTH) ? (int16_t)(X_SMP + s - S_PHARYNX0)
             : (real && s == 0)                    ? (int16_t)(X_GP + 1)
                                                   : zero;
    const int16_t esink = (int16_t)(X_OFF + EDGE_SINK);
    q.x_e0 = real && t->edge[s][0] >= 0 ? (int16_t)(X_OFF + t->edge[s][0]) : esink;
    q.x_e1 = real && t->edge[s][1] >= 0 ? (int16_t)(X_OFF + t->edge[s][1]) : esink;
    q.x_e2 = real && t->edge[s][1] >= 0 && t->edge[s][2] >= 0 ? (int16_t)(X_OFF + t->edge[s][2]) : esink;
    const int o0 = real ? t->cout0[s] : -1, o1 = real ? t->cout1[s] : -1;
    q.x_o0 = (int16_t)(X_U + (o0 >= 0 ? o0 : U_ZERO));
    q.x_o1 = (int16_t)(X_U + (o1 >= 0 ? o1 : U_ZERO));
    q.x_ur = real && c.ur_slot[s] >= 0 ? (int16_t)(X_UR + c.ur_slot[s]) : sink;
    q.x_un = real && c.un_slot[s] >= 0 ? (int16_t)(X_UN + c.un_slot[s]) : sink;
    q.x_p4 = (s >= S_LAST_TRACHEA && s <= S_PHARYNX0) ? (int16_t)(X_P4 + s - S_LAST_TRACHEA) : sink;
    q.x_uo0 = o0 >= 0 && c.un_slot[o0] >= 0 ? (int16_t)(X_UN + c.un_slot[o0]) : zero;
    q.x_uo1 = o1 >= 0 && c.un_slot[o1] >= 0 ? (int16_t)(X_UN + c.un_slot[o1]) : zero;
    for (int k = 0; k < 6; ++k) q.x_rad[k] = zero;
    if (real && (s == S_LAST_MOUTH || s == S_LAST_NOSE) && o0 >= 0 && o1 >= 0) {
      q.x_rad[0] = (int16_t)(X_U + o0);
      q.x_rad[1] = (int16_t)(X_U + o1);
      q.x_rad[2] = c.ur_slot[o0] >= 0 ? (int16_t)(X_UR + c.ur_slot[o0]) : zero;
      q.x_rad[3] = c.ur_slot[o1] >= 0 ? (int16_t)(X_UR + c.ur_slot[o1]) : zero;
      q.x_rad[4] = c.un_slot[o0] >= 0 ? (int16_t)(X_UN + c.un_slot[o0]) : zero;
      q.x_rad[5] = c.un_slot[o1] >= 0 ? (int16_t)(X_UN + c.un_slot[o1]) : zero;
    }
    q.flags = (uint16_t)((br >= 0 ? SR_BIF : 0) |
                         (real && a >= S_PHARYNX0 && s <= S_LAST_MOUTH ? SR_JUNCTION : 0) |
                         (s == S_LAST_MOUTH || s == S_LAST_NOSE ? SR_RADIATION : 0));
    // block slots -> LDS byte offsets
    for (uint16_t *f : {&q.x_la, &q.x_ra, &q.x_ea, &q.x_da, &q.x_ub, &q.x_urb, &q.x_sx, &q.x_e0, &q.x_e1,
                        &q.x_e2, &q.x_o0, &q.x_o1, &q.x_ur, &q.x_un, &q.x_p4, &q.x_uo0, &q.x_uo1})
      *f = (uint16_t)(*f * 8);
    for (int k = 0; k < 6; ++k) q.x_rad[k] = (uint16_t)(q.x_rad[k] * 8);
  }
  bank_edge_slots(c);
  for (int k = 0; k < NSTATIC; ++k) {
    int s = k < 23 ? k : k + 46;
    c.stat[k][ST_E] = t->E[s];
    c.stat[k][ST_ALPHA] = t->alpha[s];
    c.stat[k][ST_WC1] = t->wc1[s];
    c.stat[k][ST_WC2] = t->wc2[s];
    c.stat[k][ST_LW] = t->Lw[s];
    c.stat[k][ST_L] = t->L[s];
    c.stat[k][ST_R] = t->R[s];
  }
}

}  // namespace afs
