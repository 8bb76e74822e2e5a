// seg_tables.cpp -- host side of the segment-aligned kernel (seg_model.h): the lane partition,
// the per-lane records (LDS byte offsets of the utterance block) and the static condensation
// (the LDL^T of the constant static blocks, its lane-scan constants, the attach terms).
//
// The matrix entries of the static rows are the reference's (TdsModel.cpp:1785-2039 calcMatrix,
// negated as solveEquationsCholesky negates them, :2239-2253) evaluated once from the static
// section constants of afs_tables.cpp; tools/seg_solver_study.py checks the same elimination
// order in numpy against a dense solve.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "seg_model.h"

namespace afs {
namespace seg {

namespace {

// ---- the partition (seg_model.h) ------------------------------------------------------------
// dynamic lanes: four positions in walk order (-1: none) and the fold slot
const int DYN[SW][NDS] = {
    {23, 24, 25, 26, -1}, {27, 28, 29, 30, 84}, {31, 32, 33, 34, -1}, {35, 36, 37, 38, -1},
    {93, 64, 63, 62, 94}, {61, 60, 59, 58, -1}, {57, 56, 55, 54, -1}, {53, 52, 51, 50, -1},
    {49, 48, 47, 46, -1}, {45, 44, 43, 42, -1},
    {69, 68, 67, 66, -1},
    {39, 40, 41, 65, -1},  // junction lane (no walk)
    {-1, -1, -1, -1, -1}, {-1, -1, -1, -1, -1}, {-1, -1, -1, -1, -1}, {-1, -1, -1, -1, -1}};
const int ARM[SW] = {0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 2, -1, -1, -1, -1, -1};
const int FOLD_Q[SW] = {0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
// static lanes: three chain positions (far end first; -1 padding after the root) and leaves
const int STAT[SW][NSS] = {
    {0, 1, 2, -1, -1},     {3, 4, 5, -1, -1},     {6, 7, 8, -1, -1},     {9, 10, 11, -1, -1},
    {12, 13, 14, -1, -1},  {15, 16, 17, -1, -1},  {18, 19, 20, -1, -1},  {21, 22, -1, -1, -1},
    {95, 83, 82, 96, -1},  {81, 80, 79, -1, -1},  {78, 77, 76, 92, 91}, {75, 74, 73, 90, 89},
    {72, 71, 70, -1, -1},  {88, 87, 86, -1, -1},  {85, -1, -1, -1, -1}, {-1, -1, -1, -1, -1}};
const int SUBTREE[SW] = {1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 3, 3, 0};
const int ROOT_NODE[4] = {-1, 22, 70, 85}, ATTACH[4] = {-1, 23, 69, 84};

constexpr double TH1_TH = TH1 / TH;

uint16_t off(int slot) { return (uint16_t)(slot * 8); }

}  // namespace

void build_seg_tables(const Tables &t, SegTables *out) {
  std::memset(out, 0, sizeof *out);
  SegConsts &C = out->c;
  bool ok = true;
  const double idt = 1.0 / (t.dt * TH);
  auto dyn_sec = [](int s) { return s >= 23 && s <= 68; };
  auto pm = [](int s) { return s >= S_PHARYNX0 && s <= S_LAST_MOUTH; };
  const uint16_t U_ZERO = off(SX_U_ZERO), U_SINK = off(SX_U_SINK), D_ZERO = off(SX_D_ZERO),
                 D_SINK = off(SX_D_SINK), G_ZERO = off(SX_G_ZERO), G_SINK = off(SX_G_SINK), UN_SINK = off(SX_UN_SINK);
  auto p_slot = [&](int s) -> uint16_t {
    if (s >= S_LAST_TRACHEA && s <= S_PHARYNX0) return off(SX_P4 + s - S_LAST_TRACHEA);
    if (s == S_MOUTH0 + 2) return off(SX_TVP);
    if (s == S_NOSE0 + 2) return off(SX_TVP + 1);
    return U_SINK;
  };
  std::vector<int> node_uses(NC, 0);
  // where each current lives: (lane, slot, dynamic?)
  int lane_of[NC], slot_of[NC];
  bool is_dyn[NC];
  for (int c = 0; c < NC; ++c) { lane_of[c] = slot_of[c] = -1; is_dyn[c] = false; }

  // ---- dynamic slots ----
  for (int k = 0; k < SW; ++k) {
    for (int j = 0; j < NDS; ++j) {
      DynSlot &d = C.dyn[k][j];
      const int c = DYN[k][j];
      d.g_src = G_ZERO; d.g_own = G_SINK; d.d_own = D_SINK;
      d.out0 = d.out1 = U_ZERO; d.u_pub = U_SINK; d.un_pub = UN_SINK; d.p_pub = U_SINK;
      d.kind = K_NONE; d.m = 0; d.dip = 0xff; d.partner = 0xff; d.flags = 0;
      d.c0 = 1.0; d.c1 = 1.0;
      if (c < 0) continue;
      node_uses[c]++;
      lane_of[c] = k; slot_of[c] = j; is_dyn[c] = true;
      d.flags |= DF_CUR;
      d.u_pub = off(SX_U + c);
      d.un_pub = off(SX_UN + c);
      const int a = t.src[c];
      if (a < 0 || g_block(a) < 0) { ok = false; continue; }  // every dynamic row's source has a block
      d.g_src = off(g_block(a));
      const bool two = t.cout0[a] >= 0 && t.cout1[a] >= 0;
      if (c >= NS) {  // radiation current of section 64
        d.flags |= (t.cout0[a] == c) ? DF_RAD_R : DF_RAD_L;
      } else {
        const int s = c;
        d.flags |= DF_SEC;
        d.d_own = off(SX_D + s);
        if (g_block(s) < 0) ok = false;  // every dynamic slot's section has a block
        else d.g_own = off(g_block(s));
        if (j == FOLD && s != S_FOSSA0) ok = false;  // (the fold's static-section path: 84 only)
        d.out0 = t.cout0[s] >= 0 ? off(SX_U + t.cout0[s]) : U_ZERO;
        d.out1 = t.cout1[s] >= 0 ? off(SX_U + t.cout1[s]) : U_ZERO;
        d.p_pub = p_slot(s);
        if (s == S_GLOT_LO || s == S_GLOT_UP) d.flags |= DF_GLOTSEC;
        else d.flags |= DF_WALLS;
        if (pm(s)) {
          d.kind = K_PM;
          d.m = (uint8_t)(s - S_PHARYNX0);
          d.dip = (uint8_t)(s - S_PHARYNX0);
        } else if (s == S_GLOT_LO) {
          d.kind = K_GLOT0;
        } else if (s == S_GLOT_UP) {
          d.kind = K_GLOT1;
        } else if (s >= S_NOSE0 && s < S_NOSE0 + 4) {
          d.kind = K_NOSE;
          const int i = s - S_NOSE0;
          d.c0 = (double)(i * i);
        } else {  // static section behind a dynamic current (69, 84)
          d.kind = K_STATIC;
          d.c0 = t.area[s];
          d.c1 = t.len[s];
        }
        if (s == S_LAST_MOUTH) d.flags |= DF_RAD64;
        if (s == S_NOSE0 + 2) d.flags |= DF_TV67;
        if (s == S_FOSSA0) d.flags |= DF_FOSSA;
        // Bernoulli pair (a, s): pharynx/mouth, a with a single output (TdsModel.cpp:850-877)
        if (s > S_PHARYNX0 && pm(s) && pm(a) && a == s - 1 && !two) d.flags |= DF_BERN;
        if (a >= S_PHARYNX0 && s <= S_LAST_MOUTH && pm(a) && !two) d.flags |= DF_JL;  // simple rows only (:1945)
        if (c == S_GLOT_LO) d.flags |= DF_GLOT_R0;
        if (c == S_GLOT_UP) d.flags |= DF_GLOT_R1;
      }
      if (two) d.flags |= DF_BIF;
    }
    // bifurcation partners (in the lane) and the lips dipole (fold of arm B's first lane)
    for (int j = 0; j < NDS; ++j) {
      DynSlot &d = C.dyn[k][j];
      const int c = DYN[k][j];
      if (c < 0 || !(d.flags & DF_BIF)) continue;
      const int a = t.src[c];
      const int br = (t.cout0[a] == c) ? t.cout1[a] : t.cout0[a];
      for (int q = 0; q < NDS; ++q)
        if (DYN[k][q] == br) d.partner = (uint8_t)q;
      if (d.partner == 0xff) ok = false;
      // the kernel's partner pattern: slot 4 <-> 2 or 0, slot 2 <-> 4 or 3
      if (!((j == 4 && (d.partner == 2 || d.partner == 0)) || (j == 0 && d.partner == 4) ||
            (j == 2 && (d.partner == 4 || d.partner == 3)) || (j == 3 && d.partner == 2)))
        ok = false;
    }
    if (DYN[k][0] == 93) {  // the lips dipole rides on slot 0 (93 has no section, no dipole of its own)
      C.dyn[k][0].flags |= DF_LIPS;
      C.dyn[k][0].dip = (uint8_t)DIP_LIPS;
    }
    // the fold slot carries no interpolated section: a static section (84) from the tables, or none
    {
      const int f = DYN[k][FOLD];
      DynLane &Lf = C.dl[k];
      for (int q = 0; q < FK_N; ++q) Lf.fk[q] = 0.0;
      if (f >= 0 && f < NS) {
        if (!is_static_section(f)) ok = false;
        Lf.fk[FK_L] = t.L[f];
        Lf.fk[FK_R0] = t.R[f];
        Lf.fk[FK_R1] = t.R[f];
        Lf.fk[FK_E] = t.E[f];
        Lf.fk[FK_ALPHA] = t.alpha[f];
        Lf.fk[FK_K1] = t.wc1[f];
        Lf.fk[FK_K2] = t.wc2[f];
        Lf.fk[FK_K3] = t.Lw[f] * TH1_TH;
        C.dyn[k][FOLD].g_own = G_SINK;  // (nothing reads its block)
      }
      if (f >= 0 && C.dyn[k][FOLD].dip != 0xff) ok = false;
    }
    // lane record
    DynLane &L = C.dl[k];
    L.fold_q = (uint8_t)FOLD_Q[k];
    if (ARM[k] >= 0) {
      L.wf |= WF_ARM;
      if (DYN[k][1] == DYN[k][0] + 1) L.wf |= WF_ASC;
      const bool anchored = k > 0 && ARM[k - 1] == ARM[k];
      if (anchored) L.wf |= WF_ANCHOR;
      if (k + 1 == SW || ARM[k + 1] != ARM[k]) L.wf |= WF_END;
      int idx = 0;
      for (int q = k - 1; q >= 0 && ARM[q] == ARM[k]; --q) ++idx;
      L.idx = (uint8_t)idx;
      if (idx > RED_STEPS) ok = false;
      const int f = DYN[k][FOLD];
      if (f >= 0) {  // which of the fold's neighbours is its bifurcation partner
        const int a = t.src[f];
        const int br = (t.cout0[a] == f) ? t.cout1[a] : t.cout0[a];
        if (DYN[k][L.fold_q] == br) L.wf |= WF_FOLD_P0;
        else if (DYN[k][L.fold_q + 1] != br) ok = false;
        if (DYN[k][L.fold_q] != t.cin[a] && DYN[k][L.fold_q + 1] != t.cin[a]) ok = false;
      }
    } else if (k == JUNCTION_LANE) {
      L.wf |= WF_JUNCTION;
      L.idx = 0xff;
    } else {
      L.idx = 0xff;
    }
  }
  // roles fixed in the kernel
  if (!(C.dl[ARM_A_END].wf & WF_END) || !(C.dl[ARM_B_END].wf & WF_END) || !(C.dl[ARM_C_END].wf & WF_END)) ok = false;
  if (DYN[JUNCTION_LANE][0] != 39 || DYN[JUNCTION_LANE][1] != 40 || DYN[JUNCTION_LANE][2] != 41 ||
      DYN[JUNCTION_LANE][3] != 65 || DYN[ARM_A_END][3] != 38 || DYN[ARM_B_END][3] != 42 || DYN[ARM_C_END][3] != 66)
    ok = false;

  // ---- static slots ----
  for (int k = 0; k < SW; ++k) {
    StatLane &L = C.st[k];
    L.subtree = (uint8_t)SUBTREE[k];
    L.root = 0xff;
    for (int j = 0; j < NSS; ++j) {
      StatSlot &s = L.s[j];
      const int c = STAT[k][j];
      s.d_src = D_ZERO; s.d_own = D_SINK; s.out0 = s.out1 = U_ZERO; s.u_pub = U_SINK; s.un_pub = UN_SINK;
      s.p_pub = U_SINK; s.partner = 0xff; s.flags = 0; s.g_d = G_SINK;
      for (int q = 0; q < SC_N; ++q) s.c[q] = 0.0;
      s.c[SC_INVD] = 1.0;
      if (c < 0) continue;
      node_uses[c]++;
      lane_of[c] = k; slot_of[c] = j;
      s.flags |= SF_CUR;
      s.u_pub = off(SX_U + c);
      if (c == ROOT_NODE[SUBTREE[k]]) { s.flags |= SF_ROOT; L.root = (uint8_t)j; }
      const int a = t.src[c];
      const bool two = a >= 0 && t.cout0[a] >= 0 && t.cout1[a] >= 0;
      if (a >= 0) s.d_src = off(SX_D + a);
      const double La = a >= 0 ? t.L[a] : 0.0, Ra = a >= 0 ? t.R[a] : 0.0;
      double LAB = La;
      if (c < NS) {
        s.flags |= SF_SEC;
        s.d_own = off(SX_D + c);
        s.out0 = t.cout0[c] >= 0 ? off(SX_U + t.cout0[c]) : U_ZERO;
        s.out1 = t.cout1[c] >= 0 ? off(SX_U + t.cout1[c]) : U_ZERO;
        s.p_pub = p_slot(c);
        if (g_block(c) >= 0) s.g_d = off(g_block(c) + G_D);
        LAB = La + t.L[c];
        s.c[SC_E] = t.E[c];
        s.c[SC_ALPHA] = t.alpha[c];
        s.c[SC_K1] = t.wc1[c];
        s.c[SC_K2] = t.wc2[c];
        s.c[SC_K3] = t.Lw[c] * TH1_TH;
      } else {  // nostril radiation current (TdsModel.cpp:1841-1911)
        s.flags |= SF_LIPS;
        if (t.cout1[a] == c) LAB = La + t.consts.h.lrad_nose;
      }
      if (c == 0) s.flags |= SF_LUNG;
      s.c[SC_CU] = LAB * idt;
      s.c[SC_CUR] = LAB * TH1_TH;
      if (two || c >= NS) {
        const int br = (t.cout0[a] == c) ? t.cout1[a] : t.cout0[a];
        for (int q = 0; q < NSS; ++q)
          if (STAT[k][q] == br) s.partner = (uint8_t)q;
        // the kernel's partner pattern: slots 0 <-> 3, 1 <-> 4
        if (!((j == 0 && s.partner == 3) || (j == 3 && s.partner == 0) || (j == 1 && s.partner == 4) ||
              (j == 4 && s.partner == 1)))
          ok = false;
        s.c[SC_CUD] = La * idt;
        s.c[SC_CUDR] = La * TH1_TH;
      }
      (void)Ra;
    }
  }
  for (int c = 0; c < NC; ++c) ok = ok && node_uses[c] == 1;

  // ---- the static block: K in the lanes' elimination order, its LDL^T ----
  // order: lane by lane, leaves first, then the chain positions
  std::vector<int> order;
  for (int k = 0; k < SW; ++k) {
    for (int j = PS; j < NSS; ++j)
      if (STAT[k][j] >= 0) order.push_back(STAT[k][j]);
    for (int j = 0; j < PS; ++j)
      if (STAT[k][j] >= 0) order.push_back(STAT[k][j]);
  }
  const int n = (int)order.size();
  std::vector<int> pos(NC, -1);
  for (int i = 0; i < n; ++i) pos[order[i]] = i;
  // the SPD matrix A = -M over all currents, static entries only (dynamic rows are per sample)
  auto Aentry = [&](int i, int j) -> double {
    if (i == j) {
      const int a = t.src[i];
      if (i >= NS) {  // nostril radiation (rc: + Rrad, lc: + Lrad)
        const double F = t.L[a] * idt + t.R[a];
        return (t.cout0[a] == i) ? t.E[a] + F + t.consts.h.rrad_nose : t.E[a] + (t.L[a] + t.consts.h.lrad_nose) * idt + t.R[a];
      }
      const double Ea = a >= 0 ? t.E[a] : 0.0, La = a >= 0 ? t.L[a] : 0.0, Ra = a >= 0 ? t.R[a] : 0.0;
      return t.E[i] + Ea + (La + t.L[i]) * idt + (Ra + t.R[i]);
    }
    // the clique of a section: in-current / outputs
    for (int s = 0; s < NS; ++s) {
      const int m[3] = {t.cin[s], t.cout0[s], t.cout1[s]};
      bool hi = false, hj = false;
      for (int q = 0; q < 3; ++q) { hi = hi || m[q] == i; hj = hj || m[q] == j; }
      if (!hi || !hj) continue;
      const bool outs = (i == m[1] || i == m[2]) && (j == m[1] || j == m[2]);
      return outs ? t.E[s] + t.L[s] * idt + t.R[s] : -t.E[s];
    }
    return 0.0;
  };
  std::vector<double> K((size_t)n * n), Lm((size_t)n * n, 0.0), Dv(n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) K[(size_t)i * n + j] = Aentry(order[i], order[j]);
  {
    std::vector<double> W = K;
    for (int i = 0; i < n; ++i) {
      Dv[i] = W[(size_t)i * n + i];
      for (int j = i + 1; j < n; ++j) Lm[(size_t)j * n + i] = W[(size_t)j * n + i] / Dv[i];
      for (int j = i + 1; j < n; ++j) {
        const double l = Lm[(size_t)j * n + i];
        if (l == 0.0) continue;
        for (int m2 = i + 1; m2 < n; ++m2) {
          const double w = W[(size_t)i * n + m2];
          if (w == 0.0) continue;
          if (W[(size_t)j * n + m2] == 0.0 && j != m2) ok = false;  // fill outside the pattern
          W[(size_t)j * n + m2] -= l * w;
        }
      }
    }
  }
  auto lmul = [&](int a, int b) -> double {  // multiplier of predecessor b into a (0: none)
    if (a < 0 || b < 0) return 0.0;
    return Lm[(size_t)pos[a] * n + pos[b]];
  };
  // K^-1 e_r through the factorization
  auto kinv_col = [&](int r) {
    std::vector<double> v(n, 0.0);
    v[pos[r]] = 1.0;
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < i; ++j) v[i] -= Lm[(size_t)i * n + j] * v[j];
    for (int i = 0; i < n; ++i) v[i] /= Dv[i];
    for (int i = n - 1; i >= 0; --i)
      for (int j = i + 1; j < n; ++j) v[i] -= Lm[(size_t)j * n + i] * v[j];
    return v;
  };
  std::vector<double> gcol[4];
  double e_att[4] = {0, 0, 0, 0}, delta[4] = {0, 0, 0, 0};
  for (int st = 1; st <= 3; ++st) {
    gcol[st] = kinv_col(ROOT_NODE[st]);
    e_att[st] = Aentry(ROOT_NODE[st], ATTACH[st]);
    delta[st] = -e_att[st] * e_att[st] * gcol[st][pos[ROOT_NODE[st]]];
    for (double &g : gcol[st]) g *= e_att[st];
  }
  // per static lane: multipliers, corrections, scan products
  double P[SW], Pb[SW];
  for (int k = 0; k < SW; ++k) {
    StatLane &L = C.st[k];
    double *q = L.k;
    const int *sl = STAT[k];
    const bool first = !(k > 0 && SUBTREE[k - 1] == SUBTREE[k] && SUBTREE[k] != 0);
    int prev_last = -1;
    if (!first)
      for (int j = 0; j < PS; ++j)
        if (STAT[k - 1][j] >= 0) prev_last = STAT[k - 1][j];
    q[SL_FM0] = first ? 0.0 : lmul(sl[0], prev_last);
    q[SL_FM1] = lmul(sl[1], sl[0]);
    q[SL_FM2] = lmul(sl[2], sl[1]);
    q[SL_FL00] = lmul(sl[0], sl[3]);
    q[SL_FL01] = lmul(sl[1], sl[3]);
    q[SL_FL11] = lmul(sl[1], sl[4]);
    q[SL_FL12] = lmul(sl[2], sl[4]);
    q[SL_CF0] = -q[SL_FM0];
    q[SL_CF1] = -q[SL_FM1] * q[SL_CF0];
    q[SL_CF2] = -q[SL_FM2] * q[SL_CF1];
    P[k] = q[SL_CF2];
    const bool last = k + 1 < SW && SUBTREE[k + 1] == SUBTREE[k] && SUBTREE[k] != 0;
    int my_last = -1;
    for (int j = 0; j < PS; ++j)
      if (sl[j] >= 0) my_last = sl[j];
    q[SL_BM] = last ? lmul(STAT[k + 1][0], my_last) : 0.0;
    // a lane whose chain ends before position 2 has no successor but its root (no carry)
    if (last && my_last != sl[2]) ok = false;
    double cb[NSS];
    cb[2] = -q[SL_BM];
    cb[1] = -q[SL_FM2] * cb[2];
    cb[0] = -q[SL_FM1] * cb[1];
    cb[3] = -q[SL_FL00] * cb[0] - q[SL_FL01] * cb[1];
    cb[4] = -q[SL_FL11] * cb[1] - q[SL_FL12] * cb[2];
    Pb[k] = cb[0];
    for (int j = 0; j < NSS; ++j) {
      StatSlot &s = L.s[j];
      const int c = sl[j];
      s.c[SC_CB] = cb[j];
      if (c < 0) continue;
      s.c[SC_INVD] = 1.0 / Dv[pos[c]];
      s.c[SC_G] = gcol[SUBTREE[k]][pos[c]];
    }
  }
  // Hillis-Steele products: level 0 = P, level i = Q_{i-1}[k] * Q_{i-1}[k - 2^(i-1)]
  {
    double Q[SW], R[SW];
    for (int k = 0; k < SW; ++k) { Q[k] = P[k]; R[k] = Pb[k]; }
    for (int lev = 0; lev < 4; ++lev) {
      const int s = 1 << lev;
      for (int k = 0; k < SW; ++k) {
        C.st[k].k[SL_FQ0 + lev] = Q[k];
        C.st[k].k[SL_BQ0 + lev] = R[k];
      }
      double Q2[SW], R2[SW];
      for (int k = 0; k < SW; ++k) {
        Q2[k] = Q[k] * (k - s >= 0 ? Q[k - s] : 0.0);
        R2[k] = R[k] * (k + s < SW ? R[k + s] : 0.0);
      }
      for (int k = 0; k < SW; ++k) { Q[k] = Q2[k]; R[k] = R2[k]; }
    }
  }
  // attach terms on the dynamic side
  for (int st = 1; st <= 3; ++st) {
    const int d = ATTACH[st];
    const int k = lane_of[d], j = slot_of[d];
    if (k < 0 || !is_dyn[d]) { ok = false; continue; }
    DynLane &L = C.dl[k];
    if (j == 0) { L.att0 = (uint8_t)st; L.delta0 = delta[st]; L.e0 = e_att[st]; }
    else if (j == FOLD) { L.attf = (uint8_t)st; L.deltaf = delta[st]; L.ef = e_att[st]; }
    else ok = false;
    // the kernel broadcasts the roots' z from fixed lanes
    const int rl = lane_of[ROOT_NODE[st]];
    if (rl != (st == 1 ? T_ROOT_LANE : st == 2 ? N_ROOT_LANE : F_ROOT_LANE)) ok = false;
  }
  if (lane_of[23] != 0 || slot_of[23] != 0 || lane_of[69] != ARM_C_END || slot_of[69] != 0 || lane_of[84] != 1 ||
      slot_of[84] != FOLD)
    ok = false;

  // ---- edge coverage: every edge of the current graph in exactly one role ----
  {
    std::vector<int> uses((size_t)NC * NC, 0);
    auto use = [&](int a, int b) {
      if (a < 0 || b < 0) { ok = false; return; }
      if (Aentry(a, b) == 0.0 && !(a == b)) {
        // (dynamic entries are evaluated from the static tables here; a zero means no edge)
        bool edge = false;
        for (int s = 0; s < NS; ++s) {
          const int m[3] = {t.cin[s], t.cout0[s], t.cout1[s]};
          bool ha = false, hb = false;
          for (int q = 0; q < 3; ++q) { ha = ha || m[q] == a; hb = hb || m[q] == b; }
          edge = edge || (ha && hb);
        }
        if (!edge) { ok = false; return; }
      }
      uses[(size_t)std::min(a, b) * NC + std::max(a, b)]++;
    };
    for (int k = 0; k < SW; ++k) {
      if (ARM[k] >= 0) {
        for (int p = 0; p + 1 < PD; ++p) use(DYN[k][p], DYN[k][p + 1]);
        if (C.dl[k].wf & WF_ANCHOR) use(DYN[k - 1][PD - 1], DYN[k][0]);
        if (C.dl[k].wf & WF_END) use(DYN[k][PD - 1], k == ARM_A_END ? 39 : k == ARM_B_END ? 41 : 65);
        if (DYN[k][FOLD] >= 0) {
          use(DYN[k][FOLD], DYN[k][FOLD_Q[k]]);
          use(DYN[k][FOLD], DYN[k][FOLD_Q[k] + 1]);
        }
      }
      const int *sl = STAT[k];
      for (int p = 0; p + 1 < PS; ++p)
        if (sl[p] >= 0 && sl[p + 1] >= 0) use(sl[p], sl[p + 1]);
      if (C.st[k].k[SL_FM0] != 0.0) {
        int prev_last = -1;
        for (int j = 0; j < PS; ++j)
          if (STAT[k - 1][j] >= 0) prev_last = STAT[k - 1][j];
        use(prev_last, sl[0]);
      }
      if (sl[3] >= 0) { use(sl[3], sl[0]); use(sl[3], sl[1]); }
      if (sl[4] >= 0) { use(sl[4], sl[1]); use(sl[4], sl[2]); }
    }
    use(39, 40); use(40, 41); use(40, 65); use(41, 65);
    for (int st = 1; st <= 3; ++st) use(ROOT_NODE[st], ATTACH[st]);
    for (int s = 0; s < NS; ++s) {
      const int m[3] = {t.cin[s], t.cout0[s], t.cout1[s]};
      for (int x = 0; x < 3; ++x)
        for (int y = x + 1; y < 3; ++y)
          if (m[x] >= 0 && m[y] >= 0 && uses[(size_t)std::min(m[x], m[y]) * NC + std::max(m[x], m[y])] != 1) ok = false;
    }
  }

  // ---- K5's view: SX_UN offsets of every section's outputs (tree_plan.h PW_UO) ----
  for (int s = 0; s <= NS; ++s) {
    SecRec &q = out->uo[s];
    std::memset(&q, 0, sizeof q);
    const int o0 = s < NS ? t.cout0[s] : -1, o1 = s < NS ? t.cout1[s] : -1;
    q.x_uo0 = o0 >= 0 && is_dyn[o0] ? off(SX_UN + o0) : U_ZERO;
    q.x_uo1 = o1 >= 0 && is_dyn[o1] ? off(SX_UN + o1) : U_ZERO;
    // (the constriction candidates are sections 24..64: their outputs are dynamic currents)
    if (s >= S_GLOT_UP && s <= S_LAST_MOUTH && ((o0 >= 0 && !is_dyn[o0]) || (o1 >= 0 && !is_dyn[o1]))) ok = false;
  }
  // section 22: a static source of the dynamic row 23 (its D is written every sample)
  out->g22[G_L] = t.L[S_LAST_TRACHEA];
  out->g22[G_R1] = t.R[S_LAST_TRACHEA];
  out->g22[G_E] = t.E[S_LAST_TRACHEA];
  out->g22[G_AREA] = t.area[S_LAST_TRACHEA];
  out->g22[G_IAREA] = 1.0 / t.area[S_LAST_TRACHEA];
  out->g22[G_IR0] = 1.0 / std::sqrt(t.area[S_LAST_TRACHEA] / PI);
  // the walls of the dynamic sections (pharynx / mouth / nose: Tube.cpp's defaults) in the form
  // alpha = surf / K, beta = k1 w + k2 w' + k3 w'' (TdsModel.cpp:805-832 with the wall surface
  // cancelled: Lw = Mw / surf, Rw = Bw / surf, 1 / Cw = Kw / surf)
  {
    const double Mw = t.Mw[S_PHARYNX0], Bw = t.Bw[S_PHARYNX0], Kw = t.Kw[S_PHARYNX0];
    const double idt2 = 1.0 / (t.dt * t.dt * TH * TH);
    const double K = Mw * idt2 + Bw * idt + Kw;
    C.nk[NK_INVK] = 1.0 / K;
    C.nk[NK_K1] = (Mw * idt2 + Bw * idt) / K;
    C.nk[NK_K2] = (Mw * (TH1_TH + 1.0) * idt + Bw * TH1_TH) / K;
    C.nk[NK_K3] = Mw * TH1_TH / K;
    C.nk[NK_RRAD] = t.rrad_num / (9.0 * PI * PI);  // Rrad = this / A  (TdsModel.cpp:1874)
    C.nk[NK_LRAD] = t.lrad_num / (3.0 * PI);       // Lrad = this r0 / A  (:1889: 8 rho / (3 pi sqrt(A pi)))
    for (int s = S_GLOT_LO; s <= S_NOSE0 + 4; ++s)
      if (t.Mw[s] != Mw || t.Bw[s] != Bw || t.Kw[s] != Kw) ok = false;  // (one wall kind for the dynamic slots)
    if (t.Mw[S_FOSSA0] != Mw || t.Bw[S_FOSSA0] != Bw || t.Kw[S_FOSSA0] != Kw) ok = false;
  }
  (void)dyn_sec;
  out->ok = ok ? 1 : 0;
}

}  // namespace seg
}  // namespace afs
