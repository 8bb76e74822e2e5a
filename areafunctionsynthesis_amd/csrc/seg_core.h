// seg_core.h -- the segment-aligned synthesis step (seg_model.h), written once for host and
// device like tree_core.h: a phase runs on every lane of the utterance (`par`), lane-uniform
// work with LDS side effects runs in `par_uniform`'s second function (once on the CPU, on every
// lane -- identical values -- on the GPU), and cross-lane data moves by `pull` (lane gl+K's
// values, zero outside the 16-lane row), `bcast` (lane K's), `or64` and `ballot`.  On the GPU
// these are DPP row operations (seg_kernel.h); the CPU emulator (tests/emu/seg_emu.cpp) runs
// the lanes of a phase one after another.
//
// Per sample (reference stages, file:line under src/Backend):
//   block 1   Tube::interpolate (Tube.cpp:438-505), the glottis (TriangularGlottis.cpp:154-411 /
//             TwoMassModel.cpp), prepareTimeStep's section terms (TdsModel.cpp:732-1008) of every
//             slot, the dipole targets of calcNoiseSources (:1456-1604, the geometry half from
//             the K5 plan, tree_plan.h) -- the section values the rows of other lanes need go
//             to LDS (SX_G, SX_D);
//   noise     calcNoiseSample (:1630-1708): the rand() draws (glibc TYPE_3 restated) and the
//             one-pole shaping filters of the active dipoles;
//   rows      calcMatrix (:1785-2039) of every slot, from its own section (registers) and its
//             source section (one LDS gather), the Bernoulli pair terms (:850-877), the glottal
//             entrance (:898-950), the junction inductance (:1745-1778);
//   solve     the LDL^T of the same matrix (the reference: envelope Cholesky, :2231-2314):
//             the static condensation scans, the dynamic walks in registers, the arm
//             reductions and the junction by DPP;
//   update    updateVariables (:2046-2098), radiated flow and glottal tone (:687-705), the
//             output stage (Synthesizer.cpp:614-627).
#pragma once

#include <cstdint>

#include "seg_model.h"
#include "tree_core.h"

namespace afs {
namespace seg {

using tree::clampA;
using tree::D4;
using tree::fast_div;
using tree::fast_rcp;
using tree::fast_sqrt;
using tree::pivot_recip;
using tree::U4;
using tree::xat;
constexpr double THR = tree::THR;

// per-sample values of a lane (not state: cleared before a save)
struct SegWork {
  // (the section terms of block 1 go to the LDS blocks SX_G / SX_D, not to registers)
  double rrad, lrad;       // mouth radiation (the slot of section 64)
  double smp[PD];          // dipole samples (slots 0..3)
  double fD;               // D of the fold's section (84)
  // rows and the solve
  double Dp[NDS], Yp[NDS], E[NDS], Ea[NDS], ebr[NDS];  // pivot, rhs, own and source section's E
  double iv[3], Fw[3], E3[3];
  double l0, l1, il, Yl;
  double dA, yA, Ff, Db, Yb, binv, xb, Fn, xJ, ej;
  double jd[3], jy[3];     // junction lane: pivots / rhs of 39, 41, 65 after the arms' updates
  double xs[NDS];          // solution of the dynamic slots
  double sy[NSS], sz[NSS], sx[NSS];  // static: rhs, z = K^-1 y, solution
  double zc, xd;           // static condensation: z carry / the attach node's solution
  double gR0, gR1;         // glottal entrance / transition terms of section 23 (lane-uniform)
  int gon;                 // bit 0: u23 > 0, bit 1: u24 > 0
  double fl[4], p25;       // radiated flows 93..96 and the new p[25] (output stage)
  int32_t neg, pad;        // a pivot this lane met was negative (no padding bytes: SROA)
};

struct SegLane {
  // dynamic slots: section and current state
  double p[NDS], pr[NDS], w[NDS], wr[NDS], wr2[NDS];
  double u[NDS], ur[NDS];  // (the noise-smoothed flows live in SX_UN, the frame cache in SX_FC)
  double damp[PD], dout[PD], dcut[PD];  // dipoles of the slots 0..3 (the fold has none)
  uint32_t racc[PD];
  // static slots
  double sp[NSS], spr[NSS], sw[NSS], swr[NSS], swr2[NSS], su[NSS], sur[NSS];
  double sample;           // lane 0: the output of the sample
  uint64_t planw;          // word gl of this sample's plan (tree_plan.h)
  uint32_t rtmp[4];        // rand() block scratch (4th: padding)
  SegWork k;
};

// ---------------------------------------------------------------------------
// reset (Synthesizer::reset + TdsModel::resetMotion + TriangularGlottis::resetMotion)
// ---------------------------------------------------------------------------
AFS_HD inline void seg_reset_lane(SegLane &R) {
  R = SegLane{};
#pragma unroll
  for (int j = 0; j < PD; ++j) R.dcut[j] = 3000.0;
}

AFS_HD inline void seg_reset_lds(double *X, uint32_t seed) {
  for (int k = 0; k < SX_TOTAL; ++k) X[k] = 0.0;
  tree::rng_ring_seed((uint32_t *)(X + SX_RNG), seed);
}

// Launch start: the constant part of section 22's source block (its D is written every sample).
AFS_HD inline void seg_init_lds(double *X, const SegTables &S) {
  for (int q = 0; q < GB; ++q)
    if (q != G_D) X[SX_G + GB * (S_LAST_TRACHEA - G0) + q] = S.g22[q];
}

// ---------------------------------------------------------------------------
// Frame transition: cache the two frames of the interpolation.
// ---------------------------------------------------------------------------
AFS_HD inline void seg_frame_load(int gl, SegLane &R, double *X, const SegConsts &C, const afs_frame *fl,
                                  const afs_frame *fr) {
  (void)R;
  (void)C;
  for (int m = gl; m < NPM; m += SW) {  // (lanes share the 40 sections)
    double *fc = X + SX_FC + 4 * m;
    fc[0] = clampA(fl->area_cm2[m]);  // the caller's Tube stores clamped areas (Tube.cpp:337)
    fc[1] = clampA(fr->area_cm2[m]);
    fc[2] = fl->length_cm[m];
    fc[3] = fr->length_cm[m];
  }
  if (gl == 0) {
    X[SX_FRAME + 0] = fl->teeth_position_cm;
    X[SX_FRAME + 1] = fr->teeth_position_cm;
    X[SX_FRAME + 2] = clampA(fl->velum_opening_cm2);
    X[SX_FRAME + 3] = clampA(fr->velum_opening_cm2);
    for (int k = 0; k < 6; ++k) {
      X[SX_FRAME + 4 + k] = fl->glottis[k];
      X[SX_FRAME + 10 + k] = fr->glottis[k];
    }
  }
}

// Tube::interpolate of one pharynx/mouth value, not contracted into an fma, so that it is
// bit-identical to the K5 plan's geometry (tree_plan.h PlanGeom) whatever the file's flags.
AFS_HD inline double interp_area(double r1, double aL, double ratio, double aR) {
#pragma clang fp contract(off)
  return clampA(r1 * aL + ratio * aR);
}
AFS_HD inline double interp_len(double r1, double lL, double ratio, double lR) {
#pragma clang fp contract(off)
  return r1 * lL + ratio * lR;
}

// ---------------------------------------------------------------------------
// Block 1: geometry, glottis, section terms, dipole targets.
// ---------------------------------------------------------------------------
// Lane-uniform values of the sample (every lane computes the same ones).
struct SegUni {
  tree::GlotRes g;
  double dR0g, dR1g, tvsrc;
  bool on0, on1;
  tree::Target t[4];
};

template <class Xc>
AFS_HD inline void seg_targets_uniform(Xc &x, const double *X, const SegHot &T, double a_glot_up, tree::Target *t) {
  using namespace tree;
  const uint64_t hdr = x.template rec<PW_HDR>(), uo = x.template rec<PW_UO>(), uol = x.template rec<PW_UOL>();
  const uint32_t fl = (uint32_t)hdr & 0xffu;
  (void)T;
  {  // glottis: A = the upper glottis section's area (this sample's glottis), clamped at 0.1
    const double A = a_glot_up < 0.1 ? 0.1 : a_glot_up;
    const double v = narrow_flow(X, (uint32_t)(SX_UN + S_GLOT_UP + 1) * 8u, (uint32_t)SX_U_ZERO * 8u) * fast_rcp(A);
    const double full = plan_double(x.template rec<PW_GAIN_G>()) * fabs(v) * v * v * fast_sqrt(A);
    const double fdn = plan_double(x.template rec<PW_FDN + 0>());
    t[0] = Target{(uint32_t)(hdr >> 8) & 0xffu, (1.0 - fdn) * full, fdn * full, 2000.0, (fl & PF_G) != 0};
  }
#pragma unroll
  for (int c = 0; c < 2; ++c) {  // tongue constrictions (:1547-1563)
    const uint32_t o = (uint32_t)(uo >> (32 * c));
    const double invA = plan_double(c ? x.template rec<PW_T2 + 0>() : x.template rec<PW_T1 + 0>());
    const double sqA = plan_double(c ? x.template rec<PW_T2 + 1>() : x.template rec<PW_T1 + 1>());
    const double invd = plan_double(c ? x.template rec<PW_T2 + 2>() : x.template rec<PW_T1 + 2>());
    const double fdn = plan_double(c ? x.template rec<PW_FDN + 2>() : x.template rec<PW_FDN + 1>());
    const double v = narrow_flow(X, o & 0xffffu, o >> 16) * invA;
    const double fc = 0.15 * v * invd;
    const double gain = (fl & (c ? PF_T2_TEETH : PF_T1_TEETH)) ? 10.0e-7 : 5.0e-7;
    double full = gain * fabs(v) * v * v * sqA;
    if (fl & (c ? PF_T2_LAT : PF_T1_LAT)) full = 0.0;
    t[1 + c] = Target{(uint32_t)(hdr >> (16 + 8 * c)) & 0xffu, (1.0 - fdn) * full, fdn * full, clamp_fc(fc),
                      (fl & (c ? PF_T2 : PF_T1)) != 0};
  }
  {  // lower lip (:1523-1529)
    const double v = narrow_flow(X, (uint32_t)uol & 0xffffu, (uint32_t)(uol >> 16) & 0xffffu) *
                     plan_double(x.template rec<PW_L + 0>());
    const double full = 2.0e-7 * fabs(v) * v * v * plan_double(x.template rec<PW_L + 1>());
    const double fdn = plan_double(x.template rec<PW_FDN + 3>());
    t[3] = Target{(uint32_t)(hdr >> 32) & 0xffu, (1.0 - fdn) * full, fdn * full, 2000.0, (fl & PF_L) != 0};
  }
}

// The section terms of one dynamic slot (prepareTimeStep, TdsModel.cpp:732-834), with the
// divisions rewritten around one reciprocal of the area: the Poiseuille resistance of the
// circular and the elliptic section (:741-760) as polynomials in 1/A, the wall terms with the
// wall surface cancelled (alpha = surf / K, beta = k1 w + k2 w' + k3 w''; seg_tables.cpp), the
// radiation elements of section 64 (:1874, :1889) from 1/A and r0.  (Rounding-level
// differences from the reference's quotients; the decisions -- elliptic or not, the surface
// clamp -- are the reference's comparisons.)
AFS_HD inline void seg_section(SegLane &R, int j, const DynSlot &d, const Uni &U, const SegHot &T, const SegConsts &C,
                               double r1, double ratio, double open, const SegUni &su, double *X) {
  const Hot &h = T.h;
  // (the record's fields first, as values: a select whose operand is a load becomes a branch)
  const uint16_t f = d.flags;
  const int kind = d.kind;
  const double c0 = d.c0, c1 = d.c1;
  const uint16_t g_own = d.g_own, d_own = d.d_own;
  double area, len;
  {
    const double *fc = X + SX_FC + 4 * d.m;  // (section 25's for the slots that do not interpolate)
    const double apm = interp_area(r1, fc[0], ratio, fc[1]);
    const double lpm = interp_len(r1, fc[2], ratio, fc[3]);
    const double anose = clampA(open + (c0 * (h.nose4_area - open)) * (1.0 / 16));
    const bool pm = kind == K_PM, g0 = kind == K_GLOT0, g1 = kind == K_GLOT1, no = kind == K_NOSE, st = kind == K_STATIC;
    area = st ? c0 : 1.0;
    area = no ? anose : area;
    area = g1 ? su.g.go.a1 : area;
    area = g0 ? su.g.go.a0 : area;
    area = pm ? apm : area;
    len = st ? c1 : 1.0;
    len = no ? h.len_nose0 : len;
    len = g1 ? su.g.go.l1 : len;
    len = g0 ? su.g.go.l0 : len;
    len = pm ? lpm : len;
  }
  const bool glot = (f & DF_GLOTSEC) != 0;
  const double inv_area = fast_rcp(area);
  const double r0 = fast_sqrt(area * (1.0 / PI));
  const double ia2 = inv_area * inv_area;
  const bool ell = r0 < (glot ? 0.8 : 1.6);
  // elliptic: 2 mu len (a^2 + b^2) / (pi a^3 b^3), a = rmin, b = A / (pi rmin)
  //         = len / A (2 mu pi^2 rmin^2 / A^2 + 2 mu / rmin^2); circular: 4 mu pi len / A^2
  const double ce = glot ? 2.0 * MU * PI * PI * 0.64 : 2.0 * MU * PI * PI * 2.56;
  const double cf = glot ? 2.0 * MU / 0.64 : 2.0 * MU / 2.56;
  const double Rr = ell ? (len * inv_area) * fma(ce, ia2, cf) : (4.0 * MU * PI * len) * ia2;
  const double L = (RHO * 0.5 * len) * inv_area;
  const double Cc = (area * len) * (1.0 / (RHO * CSND * CSND));
  double surf = (2.0 * PI * r0) * len;
  if (surf < AMIN) surf = AMIN;
  const bool walls = U.opt.soft_walls && (f & DF_WALLS);
  const double alpha = walls ? surf * C.nk[NK_INVK] : 0.0;
  const double beta = walls ? fma(R.w[j], C.nk[NK_K1], fma(R.wr[j], C.nk[NK_K2], R.wr2[j] * C.nk[NK_K3])) : 0.0;
  const double E = fast_div(h.dt * TH, Cc + alpha);
  const double src = (f & DF_TV67) ? su.tvsrc : 0.0;
  const double D = R.p[j] + h.dtTH1 * R.pr[j] - E * (beta - src);
  const double iR0 = (PI * r0) * inv_area;  // 1 / r0
  SegWork &k = R.k;
  if (j == 1) {  // (section 64 is slot 1 of arm B's first lane) radiation R and L
    k.rrad = C.nk[NK_RRAD] * inv_area;
    k.lrad = (C.nk[NK_LRAD] * r0) * inv_area;
  }
  // the source block other lanes' rows read, and D for the static rows
  double *g = &xat(X, g_own);
  g[G_L] = L; g[G_R1] = Rr; g[G_E] = E; g[G_D] = D;
  g[G_AREA] = area; g[G_IAREA] = inv_area; g[G_IR0] = iR0; g[G_ALPHA] = alpha;
  xat(X, d_own) = D;
}

template <int MODEL, bool VARLOSS, class Xc>
AFS_HD inline void seg_block1(Xc &x, double *X, const Uni &U, const SegHot &T, const SegConsts &C, double ratio) {
  using namespace tree;
  const Hot &h = T.h;
  const afs_options &opt = U.opt;
  SegUni su;
  su.tvsrc = 0.0;
  x.par_uniform([&](int, SegLane &) {},
                [&](SegLane &) {
                  // the glottis of this sample with the previous sample's pressures p[22..25]
                  GlotIn in;
                  for (int k = 0; k < 6; ++k) { in.fl[k] = X[SX_FRAME + 4 + k]; in.fr[k] = X[SX_FRAME + 10 + k]; }
                  for (int k = 0; k < 4; ++k) in.rel[k] = X[SX_RELX + k];
                  const double p4[4] = {X[SX_P4 + 0], X[SX_P4 + 1], X[SX_P4 + 2], X[SX_P4 + 3]};
                  su.g = glottis_eval<MODEL>(in, T, ratio, p4);
                  // glottal entrance and transition terms of section 23 (TdsModel.cpp:898-950)
                  double kent = opt.glottis_loss == AFS_ENTRANCE_LOSS_VAN_DEN_BERG ? 1.375 : 1.0;
                  if constexpr (VARLOSS) {  // :1019-1039 (the filter state: identical stores)
                    const double tp = X[SX_P4 + 0] - X[SX_P4 + 3];
                    kent = fulcher_kent(iir_run<4>(X + SX_TGLOT, h.tglot_a, h.tglot_b, tp), su.g.go.a0 / 1.25);
                  }
                  const double u23 = X[SX_U + S_GLOT_LO], u24 = X[SX_U + S_GLOT_UP];
                  const double sa = h.area_last_trachea, a0 = su.g.go.a0, a1 = su.g.go.a1;
                  su.dR0g = kent * 0.5 * RHO * fabs(u23) * (fast_rcp(a0 * a0) - fast_rcp(sa * sa));
                  const double bt = (a1 < opt.flow_separation_area_ratio * a0) ? 1.0 : 0.0;
                  const double gsep = 0.8 * X[SX_GBF] + (1.0 - 0.8) * bt;
                  X[SX_GBF] = gsep;
                  su.dR1g = gsep * fabs(u24) * 0.5 * RHO * (fast_rcp(a1 * a1) - fast_rcp(a0 * a0));
                  su.on0 = u23 > 0;
                  su.on1 = u24 > 0;
                  if (opt.transvelar_coupling) {  // flow through the velum (:966-980)
                    su.tvsrc = iir_run<4>(X + SX_TVEL, h.tone_a, h.tone_b, X[SX_TVP]) +
                               iir_run<4>(X + SX_TVEL + 8, h.tvel2_a, h.tone_b, X[SX_TVP + 1]);
                  }
                });
  seg_targets_uniform(x, X, T, su.g.go.a1, su.t);
  const double r1 = 1.0 - ratio;
  const double open = r1 * X[SX_FRAME + 2] + ratio * X[SX_FRAME + 3];
  x.par([&](int gl, SegLane &R) {
#pragma unroll
    for (int j = 0; j < PD; ++j) seg_section(R, j, C.dyn[gl][j], U, T, C, r1, ratio, open, su, X);
    {  // the fold's static section (84): beta from its wall state, D; the rest are table constants
      const double *fk = C.dl[gl].fk;
      const double v = fk[FK_ALPHA] * (R.w[FOLD] * fk[FK_K1] + R.wr[FOLD] * fk[FK_K2] + R.wr2[FOLD] * fk[FK_K3]);
      const double beta = opt.soft_walls ? v : 0.0;
      const double D = R.p[FOLD] + h.dtTH1 * R.pr[FOLD] - fk[FK_E] * (beta - 0.0);
      R.k.fD = D;
      xat(X, C.dyn[gl][FOLD].d_own) = D;
    }
    // static slots: beta from the wall state, D (the other terms are table constants)
    const StatLane &S = C.st[gl];
#pragma unroll
    for (int j = 0; j < NSS; ++j) {
      const StatSlot &s = S.s[j];
      const double v = s.c[SC_ALPHA] * (R.sw[j] * s.c[SC_K1] + R.swr[j] * s.c[SC_K2] + R.swr2[j] * s.c[SC_K3]);
      const double beta = opt.soft_walls ? v : 0.0;
      const double D = R.sp[j] + h.dtTH1 * R.spr[j] - s.c[SC_E] * (beta - 0.0);
      xat(X, s.d_own) = D;
      xat(X, s.g_d) = D;  // (section 22's source block)
    }
    // the dipoles of the slots: targets in the reference's store order, the 40 Hz smoother
#pragma unroll
    for (int j = 0; j < PD; ++j) {
      const uint32_t d = C.dyn[gl][j].dip;  // 0xff: none (never targeted, never active)
      double tgt = 0.0, cut = 0.0;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const tree::Target &t = su.t[c];
        const uint32_t dn = t.up < (uint32_t)(NPM - 1) ? t.up + 1 : (uint32_t)DIP_LIPS;
        const bool hu = t.on && t.up == d, hd = t.on && dn == d;
        tgt = hu ? t.tup : tgt;
        cut = hu ? t.fc : cut;
        tgt = hd ? t.tdn : tgt;
        cut = hd ? t.fc : cut;
      }
      R.dcut[j] = cut != 0.0 ? cut : R.dcut[j];
      const double old = R.damp[j];
      const double amp = old + h.noise_amp_F * (tgt - old);
      R.damp[j] = amp;
      R.dout[j] = (old >= THR && amp < THR) ? 0.0 : R.dout[j];
      R.racc[j] = 0u;
    }
  });
  x.par_uniform([&](int, SegLane &) {},
                [&](SegLane &) {
                  for (int k = 0; k < 6; ++k) X[SX_GP + k] = su.g.gp[k];
                  for (int k = 0; k < 4; ++k) X[SX_RELX + k] = su.g.rel[k];
                });
  // (the row phase needs the glottal terms: kept in the lanes)
  x.par([&](int, SegLane &R) {
    R.k.gR0 = su.dR0g;
    R.k.gR1 = su.dR1g;
    R.k.gon = (su.on0 ? 1 : 0) | (su.on1 ? 2 : 0);
  });
}

// ---------------------------------------------------------------------------
// Noise (TdsModel.cpp:1630-1708): the rand() draws of the active dipoles (tree_core.h's
// residue-chain block generator and prefix-sum ring), the one-pole shaping filters.
// ---------------------------------------------------------------------------
template <class Xc>
AFS_HD inline void seg_rng_block(Xc &x, uint32_t *g, uint32_t *sink, int head, bool gen) {
  using namespace tree;
  constexpr int RJ = 10;
  const uint32_t b0 = g[RNG_R + ((head - 3) & (RNG_RING - 1))], b1 = g[RNG_R + ((head - 2) & (RNG_RING - 1))],
                 b2 = g[RNG_R + ((head - 1) & (RNG_RING - 1))], sb = g[RNG_S + ((head - 1) & (RNG_RING - 1))];
  x.template scan_add<3>(
      [&](int gl, SegLane &) {
        U4 v{{0u, 0u, 0u, 0u}};
        for (int c = 0; c < 3; ++c) v.v[c] = g[RNG_R + ((head + 3 * gl + c - 31) & (RNG_RING - 1))];
        return v;
      },
      [&](int gl, SegLane &R, const U4 &p) {
        const bool on = gen && gl < RJ;
        const uint32_t n0 = b0 + p.v[0], n1 = b1 + p.v[1], n2 = b2 + p.v[2];
        *(on ? &g[RNG_R + ((head + 3 * gl) & (RNG_RING - 1))] : sink) = n0;
        *(on ? &g[RNG_R + ((head + 3 * gl + 1) & (RNG_RING - 1))] : sink) = n1;
        *(on ? &g[RNG_R + ((head + 3 * gl + 2) & (RNG_RING - 1))] : sink) = n2;
        R.rtmp[0] = n0 >> 1; R.rtmp[1] = n1 >> 1; R.rtmp[2] = n2 >> 1;
      });
  x.template scan_add<1>(
      [&](int, SegLane &R) {
        U4 v{{0u, 0u, 0u, 0u}};
        v.v[0] = R.rtmp[0] + R.rtmp[1] + R.rtmp[2];
        return v;
      },
      [&](int gl, SegLane &R, const U4 &p) {
        const bool on = gen && gl < RJ;
        const uint32_t s2 = sb + p.v[0], s1 = s2 - R.rtmp[2], s0 = s1 - R.rtmp[1];
        *(on ? &g[RNG_S + ((head + 3 * gl) & (RNG_RING - 1))] : sink) = s0;
        *(on ? &g[RNG_S + ((head + 3 * gl + 1) & (RNG_RING - 1))] : sink) = s1;
        *(on ? &g[RNG_S + ((head + 3 * gl + 2) & (RNG_RING - 1))] : sink) = s2;
      });
}

template <class Xc>
AFS_HD inline void seg_noise(Xc &x, double *X, const SegHot &T, const SegConsts &C) {
  using namespace tree;
  constexpr int RNG_BLOCK = 30;
  const uint64_t act = x.or64([&](int gl, SegLane &R) {
    uint64_t m = 0;
#pragma unroll
    for (int j = 0; j < PD; ++j) {
      const uint32_t d = C.dyn[gl][j].dip;
      m |= (d < (uint32_t)NDIP && !(R.damp[j] < THR)) ? (1ull << (d & 63u)) : 0ull;
    }
    return m;
  });
  if (act == 0) {
    x.par([&](int, SegLane &R) {
#pragma unroll
      for (int j = 0; j < PD; ++j) R.k.smp[j] = 0.0;
    });
    return;
  }
  uint32_t *g = (uint32_t *)(X + SX_RNG);
  const int head0 = ((const int32_t *)g)[RNG_HEAD], pend = ((const int32_t *)g)[RNG_PEND];
  const int base = head0 - pend;
  const int need = 12 * __builtin_popcountll(act);
  auto consume = [&](int lo, int hi) {
    x.par([&](int gl, SegLane &R) {
#pragma unroll
      for (int j = 0; j < PD; ++j) {
        const uint32_t d = C.dyn[gl][j].dip;
        const uint32_t dd = d & 63u;
        const bool on = d < (uint32_t)NDIP && ((act >> dd) & 1);
        const int q0 = 12 * __builtin_popcountll(act & ((1ull << dd) - 1));
        const int a = q0 > lo ? q0 : lo, b = q0 + 12 < hi ? q0 + 12 : hi;
        const uint32_t sb = g[RNG_S + ((base + b - 1) & (RNG_RING - 1))];
        const uint32_t sa = g[RNG_S + ((base + a - 1) & (RNG_RING - 1))];
        R.racc[j] += (on && a < b) ? sb - sa : 0u;
      }
    });
  };
  int avail = pend;
  int head = head0;
  consume(0, avail);
  while (avail < need) {
    seg_rng_block(x, g, (uint32_t *)(X + SX_ACT + 8), head, true);
    x.sync();
    consume(avail, avail + RNG_BLOCK);
    avail += RNG_BLOCK;
    head = (head + RNG_BLOCK) & (RNG_RING - 1);
  }
  x.sync();
  const uint64_t ndraw = *(const uint64_t *)(X + SX_NDRAW) + (uint64_t)need;
  x.par_uniform([&](int, SegLane &) {},
                [&](SegLane &) {
                  int32_t *c = (int32_t *)g;
                  c[RNG_HEAD] = head;
                  c[RNG_PEND] = avail - need;
                  *(uint64_t *)(X + SX_NDRAW) = ndraw;
                });
  x.par([&](int gl, SegLane &R) {
#pragma unroll
    for (int j = 0; j < PD; ++j) {
      const uint32_t d = C.dyn[gl][j].dip;
      const bool on = d < (uint32_t)NDIP && ((act >> (d & 63u)) & 1);
      double xi = (double)(int32_t)R.racc[j];
      xi *= 1.0 / 2147483647.0;
      xi -= 6.0;
      xi *= 0.28867513459481288225;  // 1 / sqrt(12)
      const double cut = R.dcut[j];
      double xx = T.h.noise_x_2000;
      if (on && cut != 2000.0) xx = exp(-2.0 * PI * (cut * T.h.dt));
      double y = (1.0 - xx) * xi;
      y += xx * R.dout[j];
      R.dout[j] = on ? y : R.dout[j];
      R.k.smp[j] = on ? y * R.damp[j] : 0.0;
    }
  });
}

// rand() ahead of the next sample (tree_core.h rng_ahead): one block whenever fewer than 30
// values are pending.
template <class Xc>
AFS_HD inline void seg_rng_ahead(Xc &x, double *X) {
  using namespace tree;
  constexpr int RNG_BLOCK = 30;
  uint32_t *g = (uint32_t *)(X + SX_RNG);
  int32_t *c = (int32_t *)g;
  const int head = c[RNG_HEAD], pend = c[RNG_PEND];
  const bool gen = pend < RNG_BLOCK;
  seg_rng_block(x, g, (uint32_t *)(X + SX_ACT + 12), head, gen);
  x.par_uniform([&](int, SegLane &) {},
                [&](SegLane &) {
                  c[RNG_HEAD] = gen ? ((head + RNG_BLOCK) & (RNG_RING - 1)) : head;
                  c[RNG_PEND] = gen ? pend + RNG_BLOCK : pend;
                });
}

// ---------------------------------------------------------------------------
// Rows (calcMatrix, TdsModel.cpp:1785-2039) as the SPD matrix A = -M, y = -rhs.
// ---------------------------------------------------------------------------
// The dynamic slots: pivot, rhs, the own and source sections' E, the edge to a bifurcation
// partner (E_a + L_a / (dt theta) + R1_a).  Slots 0..3 read their own section's terms back from
// its SX_G block; the fold's section (84) is a static one (DynLane::fk, D from block 1).
AFS_HD inline void seg_rows_dyn(int gl, SegLane &R, const double *X, const Uni &U, const SegHot &T,
                                const SegConsts &C) {
  const Hot &h = T.h;
  const afs_options &opt = U.opt;
  const double idt = h.inv_dtTH;
  SegWork &k = R.k;
  const double dR0g = k.gR0, dR1g = k.gR1;
  const int onb = k.gon;
  // the source and own sections' blocks, every slot's loads first
  double sL[NDS], sR[NDS], sE[NDS], sD[NDS], sA[NDS], siR0[NDS], siA[NDS];
  double oL[NDS], oR[NDS], oE[NDS], oD[NDS], oA[NDS], oiR0[NDS], oiA[NDS];
#pragma unroll
  for (int j = 0; j < NDS; ++j) {
    const double *g = &xat(X, C.dyn[gl][j].g_src);
    sL[j] = g[G_L]; sR[j] = g[G_R1]; sE[j] = g[G_E]; sD[j] = g[G_D];
    sA[j] = g[G_AREA]; siR0[j] = g[G_IR0]; siA[j] = g[G_IAREA];
    if (j < PD) {
      const double *o = &xat(X, C.dyn[gl][j].g_own);
      oL[j] = o[G_L]; oR[j] = o[G_R1]; oE[j] = o[G_E]; oD[j] = o[G_D];
      oA[j] = o[G_AREA]; oiR0[j] = o[G_IR0]; oiA[j] = o[G_IAREA];
    }
  }
  {  // the fold's section: table constants (no Bernoulli pair, no junction term)
    const double *fk = C.dl[gl].fk;
    oL[FOLD] = fk[FK_L]; oR[FOLD] = fk[FK_R0]; oE[FOLD] = fk[FK_E]; oD[FOLD] = k.fD;
    oA[FOLD] = 1.0; oiR0[FOLD] = 0.0; oiA[FOLD] = 0.0;
  }
  // bifurcation partners (seg_tables.cpp checks the pattern: slot 4 <-> 2 or 0, slot 2 <-> 4 or 3)
  const bool p40 = C.dyn[gl][FOLD].partner == 0, p23 = C.dyn[gl][2].partner == 3;
  double uD[NDS], uDr[NDS];
  uD[0] = R.u[4]; uDr[0] = R.ur[4];
  uD[1] = 0.0; uDr[1] = 0.0;
  uD[2] = p23 ? R.u[3] : R.u[4]; uDr[2] = p23 ? R.ur[3] : R.ur[4];
  uD[3] = R.u[2]; uDr[3] = R.ur[2];
  uD[4] = p40 ? R.u[0] : R.u[2]; uDr[4] = p40 ? R.ur[0] : R.ur[2];
  const double lips = k.smp[0];  // (the lips dipole rides on slot 0 of arm B's first lane)
#pragma unroll
  for (int j = 0; j < NDS; ++j) {
    const DynSlot &d = C.dyn[gl][j];
    const uint16_t f = d.flags;
    const bool sec = (f & DF_SEC) != 0;
    const double La = sL[j], Ea = sE[j], Da = sD[j];
    const double u = R.u[j], ur = R.ur[j];
    double RA = sR[j];
    double RB = sec ? oR[j] : 0.0;
    // Bernoulli pair (source, own section) (TdsModel.cpp:850-877): R1 of the source, R0 of the own
    {
      const double Aa = sA[j], Ab = oA[j];
      const bool c = ((Ab < Aa) & (u > 0)) | ((Ab > Aa) & (u < 0));
      const bool on = (opt.turbulence_losses != 0) & ((f & DF_BERN) != 0) & c;
      const double ta = u * (0.5 * RHO) * (siA[j] * siA[j]), tb = u * (0.5 * RHO) * (oiA[j] * oiA[j]);
      RA = on ? RA - ta : RA;
      RB = on ? RB + tb : RB;
    }
    RB = ((f & DF_GLOT_R0) && (onb & 1)) ? RB + dR0g : RB;
    RA = ((f & DF_GLOT_R1) && (onb & 2)) ? RA + dR1g : RA;
    RB = ((f & DF_FOSSA) && !opt.piriform_fossa) ? h.fossa_R0 : RB;
    double LB = sec ? oL[j] : 0.0;
    LB = (f & DF_RAD_L) ? k.lrad : LB;
    RB = (f & DF_RAD_R) ? k.rrad : RB;
    double LAB = La + LB;
    if (j < PD) {  // getJunctionInductance (TdsModel.cpp:1745-1778): 8 rho H / (3 pi^2 b), H = 1 - b / a
                   // with a, b the larger and smaller radius = 8 rho / (3 pi^2) |1/r_a - 1/r_b|
      const double jl = (8.0 * RHO / (3.0 * PI * PI)) * fabs(siR0[j] - oiR0[j]);
      const bool use = (opt.inner_length_corrections != 0) & ((f & DF_JL) != 0);
      LAB = use ? LAB + jl : LAB;
    }
    const double RAB = RA + RB;
    const double EB = sec ? oE[j] : 0.0, DB = sec ? oD[j] : 0.0;
    const bool par = (f & (DF_BIF | DF_RAD_R | DF_RAD_L)) != 0;
    const double pu = par ? uD[j] : 0.0, pur = par ? uDr[j] : 0.0;
    const double S = -(((f & (DF_RAD_R | DF_RAD_L)) != 0) ? lips : (j < PD ? k.smp[j < PD ? j : 0] : 0.0));
    const double H = -idt * (LAB * u + La * pu) - (TH1 / TH) * (LAB * ur + La * pur) + S;
    const double diag = EB + Ea + (LAB * idt + RAB);
    const double rhs = H + DB - Da;
    const bool cur = (f & DF_CUR) != 0;
    k.Dp[j] = cur ? diag : 1.0;
    k.Yp[j] = cur ? -rhs : 0.0;
    k.E[j] = EB;
    k.Ea[j] = Ea;
    k.ebr[j] = Ea + (La * idt + RA);
  }
}

// The static slots: right-hand sides (the matrix is in the constants).
AFS_HD inline void seg_rows_static(int gl, SegLane &R, const double *X, const SegConsts &C, double lung,
                                   double lips) {
  const StatLane &S = C.st[gl];
  double Da[NSS], Db[NSS];
#pragma unroll
  for (int j = 0; j < NSS; ++j) {
    Da[j] = xat(X, S.s[j].d_src);
    Db[j] = xat(X, S.s[j].d_own);
  }
  // partners: slots 0 <-> 3, 1 <-> 4 (seg_tables.cpp checks the pattern)
  const double uD[NSS] = {R.su[3], R.su[4], 0.0, R.su[0], R.su[1]};
  const double uDr[NSS] = {R.sur[3], R.sur[4], 0.0, R.sur[0], R.sur[1]};
#pragma unroll
  for (int j = 0; j < NSS; ++j) {
    const StatSlot &s = S.s[j];
    const uint16_t f = s.flags;
    const double S0 = (f & SF_LUNG) ? -lung : (f & SF_LIPS) ? -lips : 0.0;
    const double H = -(s.c[SC_CU] * R.su[j] + s.c[SC_CUD] * uD[j]) - (s.c[SC_CUR] * R.sur[j] + s.c[SC_CUDR] * uDr[j]) + S0;
    const double DB = (f & SF_SEC) ? Db[j] : 0.0;
    const double rhs = H + DB - Da[j];
    R.k.sy[j] = (f & SF_CUR) ? -rhs : 0.0;
  }
}

// ---------------------------------------------------------------------------
// Solve.
// ---------------------------------------------------------------------------
// z = K^-1 y of the static slots: forward (leaves, then the chain with the carry from the
// previous lane), backward; each a local sweep, a lane scan of the carries and a correction.
template <class Xc>
AFS_HD inline void seg_static_z(Xc &x, const SegConsts &C) {
  x.par([&](int gl, SegLane &R) {
    const double *q = C.st[gl].k;
    double *y = R.k.sy;
    y[0] = y[0] - q[SL_FL00] * y[3];
    y[1] = y[1] - q[SL_FL01] * y[3] - q[SL_FL11] * y[4];
    y[2] = y[2] - q[SL_FL12] * y[4];
    y[1] = y[1] - q[SL_FM1] * y[0];
    y[2] = y[2] - q[SL_FM2] * y[1];
    R.k.zc = y[2];  // the lane's carry with a zero carry in
  });
  // inclusive scan of the carries (level products constant)
  x.template pull<-1, 1>([&](int, SegLane &R) { return D4{{R.k.zc, 0.0, 0.0, 0.0}}; },
                         [&](int gl, SegLane &R, const D4 &v) { R.k.zc += C.st[gl].k[SL_FQ0] * v.v[0]; });
  x.template pull<-2, 1>([&](int, SegLane &R) { return D4{{R.k.zc, 0.0, 0.0, 0.0}}; },
                         [&](int gl, SegLane &R, const D4 &v) { R.k.zc += C.st[gl].k[SL_FQ1] * v.v[0]; });
  x.template pull<-4, 1>([&](int, SegLane &R) { return D4{{R.k.zc, 0.0, 0.0, 0.0}}; },
                         [&](int gl, SegLane &R, const D4 &v) { R.k.zc += C.st[gl].k[SL_FQ2] * v.v[0]; });
  x.template pull<-8, 1>([&](int, SegLane &R) { return D4{{R.k.zc, 0.0, 0.0, 0.0}}; },
                         [&](int gl, SegLane &R, const D4 &v) { R.k.zc += C.st[gl].k[SL_FQ3] * v.v[0]; });
  x.template pull<-1, 1>([&](int, SegLane &R) { return D4{{R.k.zc, 0.0, 0.0, 0.0}}; },
                         [&](int gl, SegLane &R, const D4 &v) {
                           const double *q = C.st[gl].k;
                           double *y = R.k.sy;
                           const double cin = v.v[0];
                           y[0] += q[SL_CF0] * cin;
                           y[1] += q[SL_CF1] * cin;
                           y[2] += q[SL_CF2] * cin;
                           // backward with a zero carry from the next lane
                           const StatSlot *s = C.st[gl].s;
                           double *z = R.k.sz;
                           z[2] = y[2] * s[2].c[SC_INVD];
                           z[1] = y[1] * s[1].c[SC_INVD] - q[SL_FM2] * z[2];
                           z[0] = y[0] * s[0].c[SC_INVD] - q[SL_FM1] * z[1];
                           z[3] = y[3] * s[3].c[SC_INVD] - q[SL_FL00] * z[0] - q[SL_FL01] * z[1];
                           z[4] = y[4] * s[4].c[SC_INVD] - q[SL_FL11] * z[1] - q[SL_FL12] * z[2];
                           R.k.zc = z[0];
                         });
  x.template pull<1, 1>([&](int, SegLane &R) { return D4{{R.k.zc, 0.0, 0.0, 0.0}}; },
                        [&](int gl, SegLane &R, const D4 &v) { R.k.zc += C.st[gl].k[SL_BQ0] * v.v[0]; });
  x.template pull<2, 1>([&](int, SegLane &R) { return D4{{R.k.zc, 0.0, 0.0, 0.0}}; },
                        [&](int gl, SegLane &R, const D4 &v) { R.k.zc += C.st[gl].k[SL_BQ1] * v.v[0]; });
  x.template pull<4, 1>([&](int, SegLane &R) { return D4{{R.k.zc, 0.0, 0.0, 0.0}}; },
                        [&](int gl, SegLane &R, const D4 &v) { R.k.zc += C.st[gl].k[SL_BQ2] * v.v[0]; });
  x.template pull<8, 1>([&](int, SegLane &R) { return D4{{R.k.zc, 0.0, 0.0, 0.0}}; },
                        [&](int gl, SegLane &R, const D4 &v) { R.k.zc += C.st[gl].k[SL_BQ3] * v.v[0]; });
  x.template pull<1, 1>([&](int, SegLane &R) { return D4{{R.k.zc, 0.0, 0.0, 0.0}}; },
                        [&](int gl, SegLane &R, const D4 &v) {
                          const StatSlot *s = C.st[gl].s;
                          double z[NSS];
#pragma unroll
                          for (int j = 0; j < NSS; ++j) z[j] = R.k.sz[j] + s[j].c[SC_CB] * v.v[0];
#pragma unroll
                          for (int j = 0; j < NSS; ++j) R.k.sz[j] = z[j];
                          // the subtree root's z (for the attach node), selected among values
                          const int r = C.st[gl].root;
                          R.k.zc = r == 0 ? z[0] : r == 1 ? z[1] : z[2];
                        });
}

// The dynamic slots' walk: the fold, then positions 0..2 eliminated toward the boundary 3 with
// the fill edge F to the anchor (the previous lane's boundary) carried along.
AFS_HD inline void seg_walk(int gl, SegLane &R, const SegConsts &C) {
  const DynLane &L = C.dl[gl];
  SegWork &k = R.k;
  const bool arm = (L.wf & WF_ARM) != 0, asc = (L.wf & WF_ASC) != 0;
  double D[PD], Y[PD], E[PD - 1];
#pragma unroll
  for (int p = 0; p < PD; ++p) { D[p] = k.Dp[p]; Y[p] = k.Yp[p]; }
#pragma unroll
  for (int p = 0; p < PD - 1; ++p) E[p] = arm ? -(asc ? k.E[p] : k.Ea[p]) : 0.0;
  const double ea = (L.wf & WF_ANCHOR) ? -(asc ? k.Ea[0] : k.E[0]) : 0.0;
  k.ej = (L.wf & WF_END) ? -(asc ? k.E[PD - 1] : k.Ea[PD - 1]) : 0.0;
  // the fold (84 on 28/29, 94 on 93/64): its edges to the bifurcation partner (E_a + G) and to
  // the source section's in-current (-E_a)
  const bool fold = arm && (C.dyn[gl][FOLD].flags & DF_CUR);
  const double lp = fold ? k.ebr[FOLD] : 0.0, lc = fold ? -k.Ea[FOLD] : 0.0;
  const bool p0 = (L.wf & WF_FOLD_P0) != 0;
  const double l0 = p0 ? lp : lc, l1 = p0 ? lc : lp;
  const double dl = fold ? k.Dp[FOLD] : 1.0, yl = fold ? k.Yp[FOLD] : 0.0;
  const double il = pivot_recip(dl);
  bool neg = dl < 0.0;
  {
    const double f0 = l0 * il, f1 = l1 * il;
    const bool q0 = L.fold_q == 0;
    const double dq0 = fma(-f0, l0, q0 ? D[0] : D[1]), dq1 = fma(-f1, l1, q0 ? D[1] : D[2]);
    const double yq0 = fma(-f0, yl, q0 ? Y[0] : Y[1]), yq1 = fma(-f1, yl, q0 ? Y[1] : Y[2]);
    const double eq = fma(-f0, l1, q0 ? E[0] : E[1]);
    D[0] = q0 ? dq0 : D[0];
    D[1] = q0 ? dq1 : dq0;
    D[2] = q0 ? D[2] : dq1;
    Y[0] = q0 ? yq0 : Y[0];
    Y[1] = q0 ? yq1 : yq0;
    Y[2] = q0 ? Y[2] : yq1;
    E[0] = q0 ? eq : E[0];
    E[1] = q0 ? E[1] : eq;
  }
  k.l0 = l0; k.l1 = l1; k.il = il; k.Yl = yl;
  double F = ea, dA = 0.0, yA = 0.0;
#pragma unroll
  for (int p = 0; p < PD - 1; ++p) {
    const double e2 = E[p] * E[p];
    const double inv = pivot_recip(D[p]);
    neg = neg | (D[p] < 0.0);
    const double g = F * inv, hh = E[p] * inv;
    dA = fma(-g, F, dA);
    yA = fma(-g, Y[p], yA);
    D[p + 1] = fma(-e2, inv, D[p + 1]);
    Y[p + 1] = fma(-hh, Y[p], Y[p + 1]);
    k.iv[p] = inv;
    k.Fw[p] = F;
    k.E3[p] = E[p];
    k.Yp[p] = Y[p];
    F = -(g * E[p]);
  }
  k.Yp[PD - 1] = Y[PD - 1];
  k.Ff = F;
  k.Db = D[PD - 1];
  k.Yb = Y[PD - 1];
  k.dA = dA;
  k.yA = yA;
  k.neg = (neg && arm) ? 1 : 0;
}

// Back substitution of a lane's positions from its boundary's solution and the anchor's.
AFS_HD inline void seg_back(int gl, SegLane &R, const SegConsts &C, double xA) {
  SegWork &k = R.k;
  double xs[PD];
  xs[PD - 1] = k.xb;
#pragma unroll
  for (int p = PD - 2; p >= 0; --p) xs[p] = fma(-k.Fw[p], xA, fma(-k.E3[p], xs[p + 1], k.Yp[p])) * k.iv[p];
  const bool q0 = C.dl[gl].fold_q == 0;
  const double xf = fma(-k.l1, q0 ? xs[1] : xs[2], fma(-k.l0, q0 ? xs[0] : xs[1], k.Yl)) * k.il;
#pragma unroll
  for (int p = 0; p < PD; ++p) k.xs[p] = xs[p];
  k.xs[FOLD] = xf;
}

template <class Xc>
AFS_HD inline void seg_solve(Xc &x, const SegConsts &C) {
  // static: z = K^-1 y, its roots to the attach nodes (23: lane 0 slot 0, 69: lane 10 slot 0,
  // 84: lane 1 fold)
  seg_static_z(x, C);
  auto zroot = [&](int, SegLane &R) { return D4{{R.k.zc, 0.0, 0.0, 0.0}}; };
  x.template bcast<T_ROOT_LANE, 1>(zroot, [&](int, SegLane &R, const D4 &v) { R.k.jy[0] = v.v[0]; });
  x.template bcast<N_ROOT_LANE, 1>(zroot, [&](int, SegLane &R, const D4 &v) { R.k.jy[1] = v.v[0]; });
  x.template bcast<F_ROOT_LANE, 1>(zroot, [&](int, SegLane &R, const D4 &v) { R.k.jy[2] = v.v[0]; });
  x.par([&](int gl, SegLane &R) {
    const DynLane &L = C.dl[gl];
    SegWork &k = R.k;
    const double z0 = L.att0 == 1 ? k.jy[0] : L.att0 == 2 ? k.jy[1] : 0.0;
    k.Dp[0] += L.delta0;
    k.Yp[0] = fma(-L.e0, z0, k.Yp[0]);
    k.Dp[FOLD] += L.deltaf;
    k.Yp[FOLD] = fma(-L.ef, k.jy[2], k.Yp[FOLD]);
    seg_walk(gl, R, C);
  });
  // the anchors' updates go back one lane
  x.template pull<1, 2>([&](int, SegLane &R) { return D4{{R.k.dA, R.k.yA, 0.0, 0.0}}; },
                        [&](int, SegLane &R, const D4 &v) {
                          R.k.Db += v.v[0];
                          R.k.Yb += v.v[1];
                          R.k.binv = pivot_recip(R.k.Db);
                        });
  // arm reduction toward the junction: in step s the lanes at position s of their arm
  // eliminate the previous boundary (a lane off its step updates with a zero edge)
#pragma unroll
  for (int s = 1; s <= RED_STEPS; ++s) {
    x.template pull<-1, 2>([&](int, SegLane &R) { return D4{{R.k.binv, R.k.Yb, 0.0, 0.0}}; },
                           [&](int gl, SegLane &R, const D4 &v) {
                             const double Fs = (C.dl[gl].idx == s) ? R.k.Ff : 0.0;
                             const double F2 = Fs * Fs, f = Fs * v.v[0];
                             R.k.Db = fma(-F2, v.v[0], R.k.Db);
                             R.k.Yb = fma(-f, v.v[1], R.k.Yb);
                             R.k.binv = pivot_recip(R.k.Db);
                           });
  }
  x.par([&](int gl, SegLane &R) {
    R.k.neg = R.k.neg | ((((C.dl[gl].wf & WF_ARM) != 0) & (R.k.Db < 0.0)) ? 1 : 0);
    R.k.jd[0] = R.k.Dp[0];
    R.k.jy[0] = R.k.Yp[0];
    R.k.jd[1] = R.k.Dp[2];
    R.k.jy[1] = R.k.Yp[2];
    R.k.jd[2] = R.k.Dp[3];
    R.k.jy[2] = R.k.Yp[3];
  });
  // the junction lane takes the arms' last boundaries: 38 -> 39 (slot 0), 42 -> 41 (slot 2),
  // 66 -> 65 (slot 3)
  auto give = [&](int, SegLane &R) { return D4{{R.k.binv, R.k.Yb, R.k.ej, 0.0}}; };
  auto take = [&](int q) {
    return [&, q](int, SegLane &R, const D4 &v) {
      const double g = v.v[2] * v.v[0];
      R.k.jd[q] = fma(-g, v.v[2], R.k.jd[q]);
      R.k.jy[q] = fma(-g, v.v[1], R.k.jy[q]);
    };
  };
  x.template pull<ARM_A_END - JUNCTION_LANE, 3>(give, take(0));
  x.template pull<ARM_B_END - JUNCTION_LANE, 3>(give, take(1));
  x.template pull<ARM_C_END - JUNCTION_LANE, 3>(give, take(2));
  // the junction's four nodes 39, 40, 41, 65: eliminate 39, 65, 41, solve 40 (every lane runs
  // it; only the junction lane's values are used)
  x.par([&](int gl, SegLane &R) {
    SegWork &k = R.k;
    const double e01 = -k.E[0], e12 = -k.E[1], e14 = -k.E[1], e24 = k.ebr[2];
    double d0 = k.jd[0], y0 = k.jy[0], d2 = k.jd[1], y2 = k.jy[1], d4 = k.jd[2], y4 = k.jy[2];
    double d1 = k.Dp[1], y1 = k.Yp[1];
    const double i0 = pivot_recip(d0);
    const double g0 = e01 * i0;
    d1 = fma(-g0, e01, d1);
    y1 = fma(-g0, y0, y1);
    const double i4 = pivot_recip(d4);
    const double g14 = e14 * i4, g24 = e24 * i4;
    d1 = fma(-g14, e14, d1);
    y1 = fma(-g14, y4, y1);
    d2 = fma(-g24, e24, d2);
    y2 = fma(-g24, y4, y2);
    const double e12b = fma(-g14, e24, e12);
    const double i2 = pivot_recip(d2);
    const double g12 = e12b * i2;
    d1 = fma(-g12, e12b, d1);
    y1 = fma(-g12, y2, y1);
    const bool dneg = (d0 < 0.0) | (d1 < 0.0) | (d2 < 0.0) | (d4 < 0.0);
    const double x40 = dneg ? NAN : y1 * pivot_recip(d1);
    const double x41 = fma(-e12b, x40, y2) * i2;
    const double x65 = fma(-e24, x41, fma(-e14, x40, y4)) * i4;
    const double x39 = fma(-e01, x40, y0) * i0;
    const bool jn = gl == JUNCTION_LANE;
    k.jd[0] = x39; k.jd[1] = x40; k.jd[2] = x41; k.jy[0] = x65;
    (void)jn;
  });
  // back to the arms' last boundaries
  x.template pull<JUNCTION_LANE - ARM_A_END, 1>([&](int, SegLane &R) { return D4{{R.k.jd[0], 0.0, 0.0, 0.0}}; },
                                                [&](int gl, SegLane &R, const D4 &v) { R.k.xJ = gl == ARM_A_END ? v.v[0] : 0.0; });
  x.template pull<JUNCTION_LANE - ARM_B_END, 1>([&](int, SegLane &R) { return D4{{R.k.jd[2], 0.0, 0.0, 0.0}}; },
                                                [&](int gl, SegLane &R, const D4 &v) { R.k.xJ = gl == ARM_B_END ? v.v[0] : R.k.xJ; });
  x.template pull<JUNCTION_LANE - ARM_C_END, 1>([&](int, SegLane &R) { return D4{{R.k.jy[0], 0.0, 0.0, 0.0}}; },
                                                [&](int gl, SegLane &R, const D4 &v) { R.k.xJ = gl == ARM_C_END ? v.v[0] : R.k.xJ; });
  x.template pull<1, 1>([&](int, SegLane &R) { return D4{{R.k.Ff, 0.0, 0.0, 0.0}}; },
                        [&](int gl, SegLane &R, const D4 &v) {
                          R.k.Fn = v.v[0];
                          const bool end = (C.dl[gl].wf & WF_END) != 0;
                          R.k.xb = end ? fma(-R.k.ej, R.k.xJ, R.k.Yb) * R.k.binv : 0.0;
                        });
#pragma unroll
  for (int s = RED_STEPS - 1; s >= 0; --s) {
    x.template pull<1, 1>([&](int, SegLane &R) { return D4{{R.k.xb, 0.0, 0.0, 0.0}}; },
                          [&](int gl, SegLane &R, const D4 &v) {
                            const bool on = C.dl[gl].idx == s && !(C.dl[gl].wf & WF_END);
                            R.k.xb = on ? fma(-R.k.Fn, v.v[0], R.k.Yb) * R.k.binv : R.k.xb;
                          });
  }
  // a negative pivot anywhere: every solution of the sample is NaN (the reference's Cholesky
  // takes the square root of it, TdsModel.cpp:2267)
  const bool bad = x.ballot([&](int, SegLane &R) { return R.k.neg != 0; }) != 0;
  x.template pull<-1, 1>([&](int, SegLane &R) { return D4{{R.k.xb, 0.0, 0.0, 0.0}}; },
                         [&](int gl, SegLane &R, const D4 &v) {
                           seg_back(gl, R, C, v.v[0]);
                           if (gl == JUNCTION_LANE) {
                             R.k.xs[0] = R.k.jd[0];
                             R.k.xs[1] = R.k.jd[1];
                             R.k.xs[2] = R.k.jd[2];
                             R.k.xs[3] = R.k.jy[0];
                           }
#pragma unroll
                           for (int j = 0; j < NDS; ++j) R.k.xs[j] = bad ? NAN : R.k.xs[j];
                         });
  // the static slots: x = z - g x_d of their subtree's attach node
  x.template bcast<0, 1>([&](int, SegLane &R) { return D4{{R.k.xs[0], 0.0, 0.0, 0.0}}; },
                         [&](int gl, SegLane &R, const D4 &v) { R.k.xd = C.st[gl].subtree == 1 ? v.v[0] : 0.0; });
  x.template bcast<ARM_C_END, 1>([&](int, SegLane &R) { return D4{{R.k.xs[0], 0.0, 0.0, 0.0}}; },
                                 [&](int gl, SegLane &R, const D4 &v) { R.k.xd = C.st[gl].subtree == 2 ? v.v[0] : R.k.xd; });
  x.template bcast<1, 1>([&](int, SegLane &R) { return D4{{R.k.xs[FOLD], 0.0, 0.0, 0.0}}; },
                         [&](int gl, SegLane &R, const D4 &v) {
                           R.k.xd = C.st[gl].subtree == 3 ? v.v[0] : R.k.xd;
                           const StatSlot *s = C.st[gl].s;
#pragma unroll
                           for (int j = 0; j < NSS; ++j) R.k.sx[j] = fma(-s[j].c[SC_G], R.k.xd, R.k.sz[j]);
                         });
}

// ---------------------------------------------------------------------------
// Update (updateVariables, TdsModel.cpp:2046-2098) after the solution was published to SX_U.
// ---------------------------------------------------------------------------
AFS_HD inline void seg_publish_x(int gl, SegLane &R, double *X, const SegConsts &C) {
#pragma unroll
  for (int j = 0; j < NDS; ++j) xat(X, C.dyn[gl][j].u_pub) = R.k.xs[j];
#pragma unroll
  for (int j = 0; j < NSS; ++j) xat(X, C.st[gl].s[j].u_pub) = R.k.sx[j];
}

AFS_HD inline void seg_update(int gl, SegLane &R, const double *__restrict__ X, double *__restrict__ Xw, const Uni &U,
                              const SegHot &T, const SegConsts &C) {
  const double c = T.h.noise_lp_c, idt = T.h.inv_dtTH;
  // every slot's loads first: the output flows, the section's D, E, alpha (block 1, LDS)
  double o0[NDS], o1[NDS], dD[NDS], dE[NDS], dal[NDS], so0[NSS], so1[NSS], sD[NSS];
  double unold[NDS], unew[NDS];
#pragma unroll
  for (int j = 0; j < NDS; ++j) {
    const DynSlot &d = C.dyn[gl][j];
    o0[j] = xat(X, d.out0);
    o1[j] = xat(X, d.out1);
    unold[j] = xat(X, d.un_pub);
    if (j < PD) {
      const double *g = &xat(X, d.g_own);
      dD[j] = g[G_D];
      dE[j] = g[G_E];
      dal[j] = g[G_ALPHA];
    }
  }
  const double *fk = C.dl[gl].fk;
  dD[FOLD] = R.k.fD;
  dE[FOLD] = fk[FK_E];
  dal[FOLD] = U.opt.soft_walls ? fk[FK_ALPHA] : 0.0;
#pragma unroll
  for (int j = 0; j < NSS; ++j) {
    so0[j] = xat(X, C.st[gl].s[j].out0);
    so1[j] = xat(X, C.st[gl].s[j].out1);
    sD[j] = xat(X, C.st[gl].s[j].d_own);
  }
#pragma unroll
  for (int j = 0; j < NDS; ++j) {
    // beta of block 1 again, from the wall state before this update
    const bool walls = U.opt.soft_walls && (C.dyn[gl][j].flags & DF_WALLS);
    const double bd = fma(R.w[j], C.nk[NK_K1], fma(R.wr[j], C.nk[NK_K2], R.wr2[j] * C.nk[NK_K3]));
    const double bf = fk[FK_ALPHA] * (R.w[j] * fk[FK_K1] + R.wr[j] * fk[FK_K2] + R.wr2[j] * fk[FK_K3]);
    const double beta = walls ? (j < PD ? bd : bf) : 0.0;
    const double un = R.k.xs[j];
    const double uold = R.u[j];
    R.u[j] = un;
    R.ur[j] = (un - uold) * idt - (TH1 / TH) * R.ur[j];
    unew[j] = (1.0 - c) * un + c * unold[j];
    double cout = 0.0;
    cout += o0[j];
    cout += o1[j];
    double cin = 0.0;
    cin += un;
    const double net = cin - cout;
    const double old = R.p[j];
    const double p = dD[j] + dE[j] * net;
    R.p[j] = p;
    const double prr = (p - old) * idt - R.pr[j] * (TH1 / TH);
    R.pr[j] = prr;
    const double ow = R.w[j], owr = R.wr[j];
    const double w = prr * dal[j] + beta;
    R.w[j] = w;
    const double wr = (w - ow) * idt - owr * (TH1 / TH);
    R.wr[j] = wr;
    R.wr2[j] = (wr - owr) * idt - R.wr2[j] * (TH1 / TH);
  }
#pragma unroll
  for (int j = 0; j < NSS; ++j) {
    const StatSlot &s = C.st[gl].s[j];
    const double v = s.c[SC_ALPHA] * (R.sw[j] * s.c[SC_K1] + R.swr[j] * s.c[SC_K2] + R.swr2[j] * s.c[SC_K3]);
    const double beta = U.opt.soft_walls ? v : 0.0;  // (block 1's)
    const double un = R.k.sx[j];
    const double uold = R.su[j];
    R.su[j] = un;
    R.sur[j] = (un - uold) * idt - (TH1 / TH) * R.sur[j];
    double cout = 0.0;
    cout += so0[j];
    cout += so1[j];
    double cin = 0.0;
    cin += un;
    const double net = cin - cout;
    const double old = R.sp[j];
    const double p = sD[j] + s.c[SC_E] * net;
    R.sp[j] = p;
    const double prr = (p - old) * idt - R.spr[j] * (TH1 / TH);
    R.spr[j] = prr;
    const double ow = R.sw[j], owr = R.swr[j];
    const double w = prr * s.c[SC_ALPHA] + beta;
    R.sw[j] = w;
    const double wr = (w - ow) * idt - owr * (TH1 / TH);
    R.swr[j] = wr;
    R.swr2[j] = (wr - owr) * idt - R.swr2[j] * (TH1 / TH);
  }
  // publish: noise-smoothed flows (the constriction phase), p[22..25], p[43], p[67]
#pragma unroll
  for (int j = 0; j < NDS; ++j) {
    xat(Xw, C.dyn[gl][j].un_pub) = unew[j];
    xat(Xw, C.dyn[gl][j].p_pub) = R.p[j];
  }
#pragma unroll
  for (int j = 0; j < NSS; ++j) xat(Xw, C.st[gl].s[j].p_pub) = R.sp[j];
}

// The output stage (Synthesizer.cpp:614-627) as tree_core.h's, on this layout.
AFS_HD inline double seg_output_filter_one(double *X, const SegHot &T, double flow) {
  double op = (flow - X[SX_PREVFLOW]) * T.h.inv_dt;
  X[SX_PREVFLOW] = flow;
  double y = tree::iir_run<8>(X + SX_OUTF, T.h.out_a, T.h.out_b, op);
  double smp = y * 0.004;
  smp = smp * (1.0 / 32767);
  if (!isfinite(smp)) X[SX_NONFIN] = 1.0;
  return smp;
}

AFS_HD inline void seg_output_filter_run(double *X, const SegHot &T, double *o, int n) {
  double sx[8], sy[8], ca[9], cb[9];
#pragma unroll
  for (int k = 0; k < 8; ++k) { sx[k] = X[SX_OUTF + k]; sy[k] = X[SX_OUTF + 8 + k]; }
#pragma unroll
  for (int k = 0; k <= 8; ++k) { ca[k] = T.h.out_a[k]; cb[k] = T.h.out_b[k]; }
  const double inv_dt = T.h.inv_dt;
  double prev = X[SX_PREVFLOW];
  bool nonfin = false;
  double f[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = (i < n) ? o[i] : 0.0;
  for (int t0 = 0; t0 < n; t0 += 8) {
    double g[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) g[i] = (t0 + 8 + i < n) ? o[t0 + 8 + i] : 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (t0 + i >= n) break;
      const double op = (f[i] - prev) * inv_dt;
      prev = f[i];
      double acc = ca[0] * op;
#pragma unroll
      for (int k = 1; k <= 8; ++k) {
        acc += ca[k] * sx[k - 1];
        acc += cb[k] * sy[k - 1];
      }
#pragma unroll
      for (int k = 7; k > 0; --k) { sx[k] = sx[k - 1]; sy[k] = sy[k - 1]; }
      sx[0] = op;
      sy[0] = acc;
      double smp = acc * 0.004;
      smp = smp * (1.0 / 32767);
      nonfin = nonfin || !isfinite(smp);
      o[t0 + i] = smp;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = g[i];
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) { X[SX_OUTF + k] = sx[k]; X[SX_OUTF + 8 + k] = sy[k]; }
  X[SX_PREVFLOW] = prev;
  if (nonfin) X[SX_NONFIN] = 1.0;
}

// ---------------------------------------------------------------------------
// One audio sample.
// ---------------------------------------------------------------------------
template <int MODEL, class Xc>
AFS_HD inline void seg_sample_step(Xc &x, double *X, const Uni &U, const SegHot &T, const SegConsts &C, double ratio,
                                   bool defer_out) {
  if (U.opt.glottis_loss == AFS_ENTRANCE_LOSS_VARIABLE) seg_block1<MODEL, true>(x, X, U, T, C, ratio);
  else seg_block1<MODEL, false>(x, X, U, T, C, ratio);
  x.sync();
  x.mark(0);
  if (U.opt.generate_noise_sources) {
    seg_noise(x, X, T, C);
  } else {
    x.par([&](int, SegLane &R) {
#pragma unroll
      for (int j = 0; j < PD; ++j) R.k.smp[j] = 0.0;
    });
  }
  x.mark(1);
  const double lung = X[SX_GP + 1];
  // the lips sample for the nostril radiation rows: slot 0 of arm B's first lane
  x.template bcast<4, 1>([&](int, SegLane &R) { return D4{{R.k.smp[0], 0.0, 0.0, 0.0}}; },
                         [&](int gl, SegLane &R, const D4 &v) {
                           seg_rows_dyn(gl, R, X, U, T, C);
                           seg_rows_static(gl, R, X, C, lung, v.v[0]);
                         });
  x.mark(2);
  seg_solve(x, C);
  x.mark(3);
  x.par([&](int gl, SegLane &R) { seg_publish_x(gl, R, X, C); });
  // radiated flow: 93, 94 (arm B's first lane: slot 0, fold), 95, 96 (static lane 8: slot 0, leaf 0)
  x.template bcast<4, 2>([&](int, SegLane &R) { return D4{{R.k.xs[0], R.k.xs[FOLD], 0.0, 0.0}}; },
                         [&](int, SegLane &R, const D4 &v) { R.k.fl[0] = v.v[0]; R.k.fl[1] = v.v[1]; });
  x.template bcast<8, 2>([&](int, SegLane &R) { return D4{{R.k.sx[0], R.k.sx[3], 0.0, 0.0}}; },
                         [&](int, SegLane &R, const D4 &v) { R.k.fl[2] = v.v[0]; R.k.fl[3] = v.v[1]; });
  x.sync();
  seg_rng_ahead(x, X);
  x.par([&](int gl, SegLane &R) { seg_update(gl, R, X, X, U, T, C); });
  // the glottal tone filter's input: the new pressure of section 25 (lane 0, slot 2)
  x.template bcast<0, 1>([&](int, SegLane &R) { return D4{{R.p[2], 0.0, 0.0, 0.0}}; },
                         [&](int, SegLane &R, const D4 &v) { R.k.p25 = v.v[0]; });
  x.par_uniform([&](int, SegLane &) {},
                [&](SegLane &R) {
                  double flow = 0.0;
                  flow += R.k.fl[0];
                  flow += R.k.fl[1];
                  flow += R.k.fl[2];
                  flow += R.k.fl[3];
                  const double tone = tree::iir_run<4>(X + SX_TONE, T.h.tone_a, T.h.tone_b, R.k.p25);
                  flow += U.opt.radiation_from_skin ? tone : 0.0;
                  R.sample = defer_out ? flow : seg_output_filter_one(X, T, flow);
                });
  x.sync();
  x.mark(4);
}

}  // namespace seg
}  // namespace afs
