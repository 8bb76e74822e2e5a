// tree_core.h -- the cooperative ("tree") synthesis step, written once for host and device.
//
// W lanes cooperate on one utterance (W = 16 on MI355X: four utterances per wave64).
// Each lane owns ND dynamic sections (23..68: glottis, pharynx/mouth, velum taper) and
// NST static ones (trachea, nose, fossa, sinuses) with their in-currents; the persistent
// state of those sections/currents (pressure, wall motion, flows) lives in the lane's
// registers for the whole utterance.  Lanes exchange neighbour data through a per-utterance
// LDS block.  The per-sample system is solved with a fill-free leaf-first LDL^T whose four
// independent chains are eliminated by four lanes in lock step (schedule in Tables).
//
// The step is a sequence of phases.  A phase either runs on every lane (`par`), on the
// utterance's lane 0 (`one`) or on the first k lanes (`lanes`), and phases are separated
// by `sync()`.  Phases only read LDS data written by earlier phases, so the same code runs
//   * on the GPU: one lane per thread, sync() = wave-level memory barrier (tds_tree.hip),
//   * on the CPU: the W lanes of a phase one after another (tests/emu, test-only), which
//     lets the decomposition be checked against the oracle without a GPU.
//
// Reference stages restated here (file:line under src/Backend): Tube::interpolate
// Tube.cpp:438-505; TriangularGlottis::calcGeometry/incTime TriangularGlottis.cpp:154-397;
// TdsModel::prepareTimeStep TdsModel.cpp:718-1010 (noise :1188-1708); calcMatrix
// :1785-2039; solve :2231-2314 (replaced by the tree LDL^T of the same matrix);
// updateVariables :2046-2098; radiated flow :687-705; output stage Synthesizer.cpp:614-627.
#pragma once

#include <cstdint>

#if !defined(__HIPCC__)
#include <cmath>
using std::exp;
using std::fabs;
using std::isfinite;
using std::pow;
using std::sqrt;
#endif

#include "afs_model.h"

namespace afs {
namespace tree {

constexpr int DYN0 = 23;     // first dynamic section
constexpr int NDYNS = 46;    // sections 23..68
constexpr int NSTATS = 47;   // sections 0..22, 69..92
constexpr double THR = 0.001;  // MIN_DIPOLE_AMP (TdsModel.cpp:1611)

// ---------------------------------------------------------------------------
// Per-utterance LDS block (doubles).  Regions marked (n) are scratch of the noise phases
// and alias the solver arrays, which are only live from the row phase on.
// ---------------------------------------------------------------------------
enum : int {
  X_U = 0, X_UR = X_U + NC, X_UN = X_UR + NC,           // currents; 93..96 are persistent
  X_P4 = X_UN + NC,                                      // p[22], p[23], p[24], p[25]
  X_E = X_P4 + 4, X_D = X_E + NS,                        // per section
  X_L = X_D + NS, X_R1 = X_L + NDYNS, X_R0 = X_R1 + NDYNS, X_AREA = X_R0 + NDYNS,  // dynamic, s-23
  X_GLEN = X_AREA + NDYNS,                               // glottis section lengths (2)
  X_SMP = X_GLEN + 2,                                    // dipole samples (41)
  X_UNION = X_SMP + NDIP,
  //   noise scratch (n)
  X_LEN = X_UNION, X_LAT = X_LEN + NPM, X_POS = X_LAT + NPM, X_TGT = X_POS + NPM,
  X_CUTN = X_TGT + NDIP, X_ACT = X_CUTN + NDIP, X_NOISE_END = X_ACT + NDIP,
  //   solver
  X_DIAG = X_UNION, X_RHS = X_DIAG + NC, X_OFF = X_RHS + NC, X_SOLVE_END = X_OFF + TREE_NE,
  X_AFTER = (X_NOISE_END > X_SOLVE_END ? X_NOISE_END : X_SOLVE_END),
  // frame-rate values written by lane 0 at every frame transition
  X_FRAME = X_AFTER,           // teethL, teethR, velL, velR, gL[6], gR[6]
  // persistent small state
  X_RELX = X_FRAME + 16,       // glottis: cur0, cur1, prev0, prev1
  X_GBF = X_RELX + 4,
  X_TONE = X_GBF + 1,          // glottal tone filter: x1..x4, y1..y4
  X_OUTF = X_TONE + 8,         // output Chebyshev: x1..x8, y1..y8
  X_PREVFLOW = X_OUTF + 16,
  X_NONFIN = X_PREVFLOW + 1,
  X_ART = X_NONFIN + 1,        // 40 articulator bytes
  X_RNG = X_ART + 5,           // 31 int32 words + ring index (16 doubles)
  X_GP = X_RNG + 16,           // interpolated glottis controls (6) and teeth position (lane 0)
  X_TOTAL = X_GP + 8
};

template <int W>
struct Shape {
  static constexpr int ND = (NDYNS + W - 1) / W;
  static constexpr int NST = (NSTATS + W - 1) / W;
  static constexpr int NSL = ND + NST;
  static constexpr int NDP = (NDIP + W - 1) / W;
};

AFS_HD inline int dyn_section(int W, int j, int gl) {
  int k = j * W + gl;
  return k < NDYNS ? DYN0 + k : -1;
}
AFS_HD inline int static_section(int W, int j, int gl) {
  int k = j * W + gl;
  return k < NSTATS ? (k < 23 ? k : k + 46) : -1;
}

// Lane registers.
// Only the persistent state and the frame cache live here; per-sample intermediates
// go through the LDS block or are recomputed from unchanged state.
template <int W>
struct Lane {
  using S = Shape<W>;
  double p[S::NSL], pr[S::NSL], w[S::NSL], wr[S::NSL], wr2[S::NSL];  // sections
  double u[S::NSL], ur[S::NSL], un[S::NSL];                          // their in-currents
  double aL[S::ND], aR[S::ND], lL[S::ND], lR[S::ND], tL[S::ND], tR[S::ND];  // frame cache
  double al[S::ND], be[S::ND];                                        // dynamic wall terms
  double damp[S::NDP], dout[S::NDP], dcut[S::NDP];                   // dipoles gl + k W
  double rad_u[2], rad_ur[2], rad_un[2];                             // owner of 64 / 83
  double sample;                                                     // lane 0
  int art[S::ND];
};

template <int W>
AFS_HD inline int slot_section(int j, int gl) {
  return j < Shape<W>::ND ? dyn_section(W, j, gl) : static_section(W, j - Shape<W>::ND, gl);
}

// ---------------------------------------------------------------------------
// math helpers
// ---------------------------------------------------------------------------
AFS_HD inline double clampA(double a) { return a < AMIN ? AMIN : a; }

AFS_HD inline double glottis_q(double f0) {
  double q = 1.0 + (f0 - G_NAT_F0) / G_F0_DIV_Q;
  return q < 0.05 ? 0.05 : q;
}

// getOpenCloseDimensions (TriangularGlottis.cpp:474-576)
AFS_HD inline void glottis_open_close(const double *gp, double cord, double rel0, double rel1,
                                      double *olen, double *clen, double *ow, double *cz) {
  const double rest[2] = {gp[2], gp[3]};
  const double rel[2] = {rel0, rel1};
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    double back = rest[i] + rel[i];
    double front = (rest[i] < 0.0) ? back : rel[i];
    olen[i] = 0.0; ow[i] = 0.0; clen[i] = cord; cz[i] = 0.5 * cord;
    if (back > 0.0 && front > 0.0) {
      olen[i] = cord; ow[i] = back + front; clen[i] = 0.0; cz[i] = 0.0;
    } else if (back <= 0.0 && front <= 0.0) {
      olen[i] = 0.0; ow[i] = 0.0; clen[i] = cord; cz[i] = 0.5 * cord;
    } else {
      double r = rest[i];
      if (fabs(r) < 0.000000001) r = 0.000000001;
      double apex = cord * (1.0 + rel[i] / r);
      if (apex >= 0.0 && apex <= cord) {
        if (back > 0.0) {
          olen[i] = apex; ow[i] = back; clen[i] = cord - apex; cz[i] = 0.5 * (apex + cord);
        } else {
          olen[i] = cord - apex; ow[i] = front; clen[i] = apex; cz[i] = 0.5 * apex;
        }
      }
    }
  }
}

// getJunctionInductance (TdsModel.cpp:1745-1778)
AFS_HD inline double junction_l(double A1, double A2) {
  if (A1 < AMIN) A1 = AMIN;
  if (A2 < AMIN) A2 = AMIN;
  double a, b;
  if (A1 > A2) { a = sqrt(A1 / PI); b = sqrt(A2 / PI); }
  else { a = sqrt(A2 / PI); b = sqrt(A1 / PI); }
  double H = 1.0 - b / a;
  return 8.0 * RHO * H / (3.0 * PI * PI * b);
}

// IirFilter::getOutputSample on a shift-register state x[0..n-1], y[0..n-1] (newest first)
AFS_HD inline double iir_run(double *st, int n, const double *a, const double *b, double x) {
  double acc = a[0] * x;
  for (int k = 1; k <= n; ++k) {
    acc += a[k] * st[k - 1];
    acc += b[k] * st[n + k - 1];
  }
  for (int k = n - 1; k > 0; --k) { st[k] = st[k - 1]; st[n + k] = st[n + k - 1]; }
  st[0] = x;
  st[n] = acc;
  return acc;
}

AFS_HD inline int32_t rng_next(int32_t *r) {
  int f = r[31];
  int q = f - 3;
  if (q < 0) q += 31;
  uint32_t v = (uint32_t)r[f] + (uint32_t)r[q];
  r[f] = (int32_t)v;
  r[31] = (f + 1 == 31) ? 0 : f + 1;
  return (int32_t)(v >> 1);
}

// glibc __srandom_r: Schrage fill + 310 discarded outputs
AFS_HD inline void rng_seed(int32_t *r, uint32_t seed) {
  if (seed == 0) seed = 1;
  int32_t word = (int32_t)seed;
  r[0] = word;
  for (int i = 1; i < 31; ++i) {
    long long hi = word / 127773;
    long long lo = word % 127773;
    long long nw = 16807 * lo - 2836 * hi;
    if (nw < 0) nw += 2147483647;
    word = (int32_t)nw;
    r[i] = word;
  }
  r[31] = 3;
  for (int k = 0; k < 310; ++k) (void)rng_next(r);
}

// ---------------------------------------------------------------------------
// Reset (Synthesizer::reset + TdsModel::resetMotion + TriangularGlottis::resetMotion)
// ---------------------------------------------------------------------------
template <int W>
AFS_HD inline void reset_lane(int gl, Lane<W> &R) {
  using S = Shape<W>;
  (void)gl;
#pragma unroll
  for (int j = 0; j < S::NSL; ++j) {
    R.p[j] = R.pr[j] = R.w[j] = R.wr[j] = R.wr2[j] = 0.0;
    R.u[j] = R.ur[j] = R.un[j] = 0.0;
  }
#pragma unroll
  for (int j = 0; j < S::ND; ++j) {
    R.aL[j] = R.aR[j] = R.lL[j] = R.lR[j] = R.tL[j] = R.tR[j] = R.al[j] = R.be[j] = 0.0;
    R.art[j] = OTHER;
  }
#pragma unroll
  for (int k = 0; k < S::NDP; ++k) { R.damp[k] = 0.0; R.dout[k] = 0.0; R.dcut[k] = 3000.0; }
  for (int k = 0; k < 2; ++k) R.rad_u[k] = R.rad_ur[k] = R.rad_un[k] = 0.0;
  R.sample = 0.0;
}

AFS_HD inline void reset_lds(double *X, uint32_t seed) {
  for (int k = 0; k < X_TOTAL; ++k) X[k] = 0.0;
  rng_seed((int32_t *)(X + X_RNG), seed);
}

// ---------------------------------------------------------------------------
// Frame transition: cache the two frames of the interpolation.
// ---------------------------------------------------------------------------
template <int W>
AFS_HD inline void frame_load(int gl, Lane<W> &R, double *X, const afs_frame *fl, const afs_frame *fr) {
  using S = Shape<W>;
#pragma unroll
  for (int j = 0; j < S::ND; ++j) {
    int s = dyn_section(W, j, gl);
    int m = s - S_PHARYNX0;
    if (m >= 0 && m < NPM) {
      R.aL[j] = clampA(fl->area_cm2[m]);   // the caller's Tube stores clamped areas (Tube.cpp:337)
      R.aR[j] = clampA(fr->area_cm2[m]);
      R.lL[j] = fl->length_cm[m];
      R.lR[j] = fr->length_cm[m];
      R.tL[j] = fl->laterality[m];
      R.tR[j] = fr->laterality[m];
      R.art[j] = fl->articulator[m];       // articulator comes from the left tube (Tube.cpp:452)
    }
  }
  if (gl == 0) {
    X[X_FRAME + 0] = fl->teeth_position_cm;
    X[X_FRAME + 1] = fr->teeth_position_cm;
    X[X_FRAME + 2] = clampA(fl->velum_opening_cm2);   // getVelumOpening = clamped noseSection[0]
    X[X_FRAME + 3] = clampA(fr->velum_opening_cm2);
    for (int k = 0; k < 6; ++k) {
      X[X_FRAME + 4 + k] = fl->glottis[k];
      X[X_FRAME + 10 + k] = fr->glottis[k];
    }
    unsigned char *art = (unsigned char *)(X + X_ART);
    for (int m = 0; m < NPM; ++m) art[m] = fl->articulator[m];
  }
}

// ---------------------------------------------------------------------------
// Phase G: tube interpolation (all lanes) and the glottis (lane 0).
// ---------------------------------------------------------------------------
template <int W>
AFS_HD inline void phase_geometry(int gl, Lane<W> &R, double *X, const Tables &T, double ratio) {
  using S = Shape<W>;
  const double r1 = 1.0 - ratio;
#pragma unroll
  for (int j = 0; j < S::ND; ++j) {
    const int s = dyn_section(W, j, gl);
    if (s >= S_PHARYNX0 && s <= S_LAST_MOUTH) {
      X[X_AREA + s - DYN0] = clampA(r1 * R.aL[j] + ratio * R.aR[j]);
      X[X_LEN + s - S_PHARYNX0] = r1 * R.lL[j] + ratio * R.lR[j];
      X[X_LAT + s - S_PHARYNX0] = r1 * R.tL[j] + ratio * R.tR[j];
    } else if (s >= S_NOSE0) {  // nose sections 65..68: velum taper (Tube.cpp:402-416)
      double open = r1 * X[X_FRAME + 2] + ratio * X[X_FRAME + 3];
      int i = s - S_NOSE0;
      X[X_AREA + s - DYN0] = clampA(open + ((double)(i * i) * (T.nose4_area - open)) / (double)16);
    }
  }
  if (gl == 0) {
    double gp[6];
    for (int k = 0; k < 6; ++k) {
      gp[k] = r1 * X[X_FRAME + 4 + k] + ratio * X[X_FRAME + 10 + k];
      X[X_GP + k] = gp[k];
    }
    X[X_GP + 6] = r1 * X[X_FRAME + 0] + ratio * X[X_FRAME + 1];
    double rel0 = X[X_RELX + 0], rel1 = X[X_RELX + 1];
    // calcGeometry + getTubeData + Tube::setGlottisGeometry (TriangularGlottis.cpp:338-411)
    double chink = gp[4] < 0.0 ? 0.0 : gp[4];
    double q = glottis_q(gp[0]);
    double f = sqrt(q);
    double cord = G_REST_LEN * f;
    double th0 = G_REST_THICK0 / f, th1 = G_REST_THICK1 / f;
    double olen[2], clen[2], ow[2], cz[2];
    glottis_open_close(gp, cord, rel0, rel1, olen, clen, ow, cz);
    X[X_AREA + 0] = clampA(olen[0] * ow[0] + chink);
    X[X_AREA + 1] = clampA(olen[1] * ow[1] + chink);
    X[X_GLEN + 0] = th0;
    X[X_GLEN + 1] = th1;
    // incTime (TriangularGlottis.cpp:154-330) with the previous sample's pressures
    const double Tt = 1.0 / T.fs;
    const double p0 = X[X_P4 + 0], p1 = X[X_P4 + 1], p2 = X[X_P4 + 2], p3 = X[X_P4 + 3];
    double m0 = G_MASS0 / q, m1 = G_MASS1 / q;
    double al0 = clen[0] / cord, al1 = clen[1] / cord;
    double k0 = G_K0 * q, k1 = G_K1 * q, kc0 = G_KC0 * q, kc1 = G_KC1 * q;
    double kcp = G_KCOUPLE * q * q;
    double dr0 = G_DAMP0 + al0 * 1.0, dr1 = G_DAMP1 + al1 * 1.0;
    double rr0 = 2.0 * dr0 * sqrt(m0 * k0), rr1 = 2.0 * dr1 * sqrt(m1 * k1);
    double fo0 = p1 * olen[0] * th0;
    double fo1 = p2 * olen[1] * th1;
    fo0 += 0.5 * 0.5 * (p0 + p1) * G_INLET * cord;
    fo1 += 0.5 * 0.5 * (p3 + p2) * G_OUTLET * cord;
    double rs0 = (gp[2] >= 0.0) ? gp[2] * (1.0 - cz[0] / cord) : gp[2];
    double rs1 = (gp[3] >= 0.0) ? gp[3] * (1.0 - cz[1] / cord) : gp[3];
    double A = m0 + rr0 * Tt + Tt * Tt * (k0 + kc0 * al0) + kcp * Tt * Tt;
    double B = -kcp * Tt * Tt;
    double Cq = -kcp * Tt * Tt;
    double Dq = m1 + rr1 * Tt + Tt * Tt * (k1 + kc1 * al1) + kcp * Tt * Tt;
    double Ee = fo0 * Tt * Tt + 2.0 * m0 * rel0 - m0 * X[X_RELX + 2] + rr0 * Tt * rel0 - Tt * Tt * kc0 * al0 * rs0;
    double Ff = fo1 * Tt * Tt + 2.0 * m1 * rel1 - m1 * X[X_RELX + 3] + rr1 * Tt * rel1 - Tt * Tt * kc1 * al1 * rs1;
    double det = A * Dq - B * Cq;
    if (fabs(det) < 0.000000001) det = 0.000000001;
    X[X_RELX + 2] = rel0;
    X[X_RELX + 3] = rel1;
    X[X_RELX + 0] = (Ee * Dq - B * Ff) / det;
    X[X_RELX + 1] = (A * Ff - Ee * Cq) / det;
  }
}

// ---------------------------------------------------------------------------
// Phase N: per-section network elements L, C, R, wall terms, D, E (TdsModel.cpp:732-1008).
// Static sections take L, C, R, alpha, E from the tables; only beta and D depend on state.
// ---------------------------------------------------------------------------
AFS_HD inline int static_index(int s) { return s < 23 ? s : s - 46; }

template <int W>
AFS_HD inline double static_beta(const Lane<W> &R, int j, const Tables &T, const Consts &C, int s) {
  const double *k = C.stat[static_index(s)];
  return T.opt.soft_walls ? k[ST_ALPHA] * (R.w[j] * k[ST_WC1] + R.wr[j] * k[ST_WC2] + R.wr2[j] * k[ST_LW] * (TH1 / TH))
                          : 0.0;
}

template <int W>
AFS_HD inline void phase_network(int gl, Lane<W> &R, double *X, const Tables &T, const Consts &C) {
  using S = Shape<W>;
  const afs_options &opt = T.opt;
  const double dt = T.dt;
#pragma unroll
  for (int j = 0; j < S::NST; ++j) {
    const int jj = S::ND + j;
    const int s = static_section(W, j, gl);
    if (s < 0) continue;
    const double E = C.stat[static_index(s)][ST_E];
    const double beta = static_beta<W>(R, jj, T, C, s);
    X[X_E + s] = E;
    X[X_D + s] = R.p[jj] + T.dtTH1 * R.pr[jj] - E * (beta - 0.0);
  }
#pragma unroll
  for (int j = 0; j < S::ND; ++j) {
    const int s = dyn_section(W, j, gl);
    if (s < 0) continue;
    const bool glot = (s == S_GLOT_LO || s == S_GLOT_UP);
    const double area = X[X_AREA + s - DYN0];
    const double len = glot ? X[X_GLEN + s - DYN0] : (s <= S_LAST_MOUTH ? X[X_LEN + s - S_PHARYNX0] : T.len[S_NOSE0]);
    const double vol = area * len;
    double alpha = 0.0, beta = 0.0;
    double circ = 2.0 * sqrt(area * PI);
    double a = sqrt(area / PI), b = a;
    double rmin = glot ? 0.8 : 1.6;
    if (a < rmin) { a = rmin; b = area / (PI * a); }
    const double L = (RHO * 0.5 * len) / area;
    const double C = vol / (RHO * CSND * CSND);
    const double Rr = ((2.0 * MU * len) * (a * a + b * b)) / (PI * a * a * a * b * b * b);
    if (opt.soft_walls && !glot) {
      double surf = circ * len;
      if (surf < AMIN) surf = AMIN;
      double Rw = T.Bw[S_PHARYNX0] / surf, Lw = T.Mw[S_PHARYNX0] / surf, Cw = surf / T.Kw[S_PHARYNX0];
      alpha = 1.0 / (Lw / (dt * dt * TH * TH) + Rw / (dt * TH) + 1.0 / Cw);
      beta = alpha * (R.w[j] * (Lw / (dt * dt * TH * TH) + Rw / (dt * TH)) +
                      R.wr[j] * (Lw * (TH1 / TH + 1.0) / (dt * TH) + Rw * (TH1 / TH)) +
                      R.wr2[j] * Lw * (TH1 / TH));
    }
    const double E = dt * TH / (C + alpha);
    double R0 = Rr, R1 = Rr;
    // Bernoulli losses between pharynx/mouth sections (TdsModel.cpp:850-877)
    if (opt.turbulence_losses && s >= S_PHARYNX0 && s <= S_LAST_MOUTH) {
      if (s < S_LAST_MOUTH && s != S_PHARYNX0 + 3 && s != S_LAST_PHARYNX) {  // pair (s, s+1)
        double u = 0.0;
        u += X[X_U + s + 1];
        double Ai = X[X_AREA + s + 1 - DYN0];
        if ((Ai < area && u > 0) || (Ai > area && u < 0)) R1 = R1 - u * 0.5 * RHO / (area * area);
      }
      if (s > S_PHARYNX0 && s - 1 != S_PHARYNX0 + 3 && s - 1 != S_LAST_PHARYNX) {  // pair (s-1, s)
        double u = 0.0;
        u += R.u[j];
        double Aa = X[X_AREA + s - 1 - DYN0];
        if ((area < Aa && u > 0) || (area > Aa && u < 0)) R0 = R0 + u * 0.5 * RHO / (area * area);
      }
    }
    if (s == S_GLOT_LO) {  // glottal entrance and transition (TdsModel.cpp:912-950)
      double sa = T.area[S_LAST_TRACHEA], ta = area;
      double u = 0.0;
      u += R.u[j];
      if (u > 0) R0 = R0 + 1.0 * 0.5 * RHO * fabs(u) * (1.0 / (ta * ta) - 1.0 / (sa * sa));
      sa = ta;
      ta = X[X_AREA + 1];
      double bt = (ta < 1.0 * sa) ? 1.0 : 0.0;
      double g = 0.8 * X[X_GBF] + (1.0 - 0.8) * bt;
      X[X_GBF] = g;
      u = 0.0;
      u += X[X_U + S_GLOT_UP];
      if (u > 0) R1 = R1 + g * fabs(u) * 0.5 * RHO * (1.0 / (ta * ta) - 1.0 / (sa * sa));
    }
    R.al[j] = alpha;
    R.be[j] = beta;
    X[X_E + s] = E;
    X[X_D + s] = R.p[j] + T.dtTH1 * R.pr[j] - E * (beta - 0.0);
    X[X_L + s - DYN0] = L;
    X[X_R0 + s - DYN0] = R0;
    X[X_R1 + s - DYN0] = R1;
  }
  // reset the dipole targets this lane owns (calcNoiseSources, TdsModel.cpp:1203-1208)
#pragma unroll
  for (int k = 0; k < S::NDP; ++k) {
    int d = gl + k * W;
    if (d < NDIP) { X[X_TGT + d] = 0.0; X[X_CUTN + d] = 0.0; }
  }
}

// ---------------------------------------------------------------------------
// Phase C (lane 0): constriction detection and dipole targets (TdsModel.cpp:1188-1604).
// ---------------------------------------------------------------------------
struct Cons { int first, last, narrow, art; double obst, lat; };

AFS_HD inline void grow(const double *X, const unsigned char *art, Cons &c, double amin_, int a) {
  double amax = amin_ + 0.2;
  while (X[X_AREA + c.first - DYN0] < amax && art[c.first - S_PHARYNX0] == a && c.first > S_PHARYNX0) c.first--;
  while (X[X_AREA + c.last - DYN0] < amax && art[c.last - S_PHARYNX0] == a && c.last < S_LAST_MOUTH) c.last++;
  c.first++;
  c.last--;
}

AFS_HD inline void tongue_obstacle(const double *X, double teeth, Cons &c, double &min_teeth) {
  for (int i = c.first; i <= c.last; ++i) {
    double lt = X[X_LAT + i - S_PHARYNX0];
    if (lt > c.lat) c.lat = lt;
  }
  double jet = X[X_POS + c.last - S_PHARYNX0] + X[X_LEN + c.last - S_PHARYNX0];
  if (teeth - jet < 2.0) {
    c.obst = teeth;
    min_teeth = X[X_AREA + c.narrow - DYN0];
  } else {
    c.obst = X[X_POS + c.last + 1 - S_PHARYNX0] + 0.5 * X[X_LEN + c.last + 1 - S_PHARYNX0];
  }
}

// Dipole targets of one constriction (TdsModel.cpp:1456-1602).
AFS_HD inline void dipole_targets(double *X, const Tables &T, const Consts &C, double teeth, const Cons &c) {
  int ob = -1;
  for (int i = S_PHARYNX0; i <= S_LAST_MOUTH && ob == -1; ++i) {
    double pos = X[X_POS + i - S_PHARYNX0];
    if (pos <= c.obst && pos + X[X_LEN + i - S_PHARYNX0] >= c.obst) ob = i;
  }
  if (ob == -1) return;
  int up = ob - S_PHARYNX0;
  int dn = (ob < S_LAST_MOUTH) ? up + 1 : DIP_LIPS;
  double fdn = (c.obst - X[X_POS + up]) / X[X_LEN + up];
  double fup = 1.0 - fdn;
  double A = X[X_AREA + c.narrow - DYN0];
  if (A < 0.1) A = 0.1;
  double flow = 0.0;
  int o0 = C.topo[c.narrow][TP_OUT0], o1 = C.topo[c.narrow][TP_OUT1];
  if (o0 != -1) flow += X[X_UN + o0];
  if (o1 != -1) flow += X[X_UN + o1];
  if (flow < 0.0) flow = 0.0;
  double v = flow / A;
  double fc = 6000.0, gain = 0.0;
  if (c.art == LOWER_LIP) {
    gain = 2.0e-7;
  } else if (c.art == VOCAL_FOLDS) {
    gain = 0.5e-7 * pow(10.0, X[X_GP + 5] / 20.0);
  } else {
    double d = sqrt(4.0 * A / PI);
    fc = 0.15 * v / d;
    gain = (fabs(c.obst - teeth) < 0.0001) ? 10.0e-7 : 5.0e-7;
  }
  double full = gain * fabs(v) * v * v * sqrt(A);
  if (c.lat > 0.1) full = 0.0;
  if (fc < 50.0) fc = 50.0;
  if (fc > 2000.0) fc = 2000.0;
  X[X_TGT + up] = fup * full; X[X_CUTN + up] = fc;
  X[X_TGT + dn] = fdn * full; X[X_CUTN + dn] = fc;
}

template <int W>
AFS_HD inline void phase_constrictions(Lane<W> &R, double *X, const Tables &T, const Consts &C) {
  const unsigned char *art = (const unsigned char *)(X + X_ART);
  const double teeth = X[X_GP + 6];
  {  // section positions (Tube::calcPositions, Tube.cpp:611-622)
    double x = 0.0;
    for (int m = 0; m < NPM; ++m) {
      X[X_POS + m] = x;
      x += X[X_LEN + m];
    }
  }
  // Up to four constrictions in the reference's order: glottis, tongue, second tongue, lip.
  const Cons cg = Cons{S_GLOT_LO, S_GLOT_UP, S_GLOT_UP, VOCAL_FOLDS, 1.5, 0.0};
  Cons ct1 = cg, ct2 = cg, cl = cg;
  bool has_t1 = false, has_t2 = false, has_l = false;
  double min_teeth = 1000000.0, mt = 1000000.0;
  int mts = -1;
  for (int i = S_PHARYNX0; i <= S_LAST_MOUTH; ++i) {
    double a = X[X_AREA + i - DYN0];
    if (art[i - S_PHARYNX0] == TONGUE && a < mt) { mt = a; mts = i; }
  }
  if (mt < 1.0) {
    has_t1 = true;
    ct1 = Cons{mts, mts, mts, TONGUE, 0.0, 0.0};
    grow(X, art, ct1, mt, TONGUE);
    tongue_obstacle(X, teeth, ct1, min_teeth);
  }
  if (has_t1) {
    const Cons pc = ct1;
    mt = 1000000.0;
    mts = -1;
    for (int i = S_PHARYNX0; i <= S_LAST_MOUTH; ++i) {
      double a = X[X_AREA + i - DYN0];
      if (art[i - S_PHARYNX0] == TONGUE && a < mt && (i < pc.first || i > pc.last)) { mt = a; mts = i; }
    }
    if (mt < 1.0) {
      ct2 = Cons{mts, mts, mts, TONGUE, 0.0, 0.0};
      grow(X, art, ct2, mt, TONGUE);
      if (ct2.first > pc.last + 1 || ct2.last < pc.first - 1) {
        has_t2 = true;
        tongue_obstacle(X, teeth, ct2, min_teeth);
      }
    }
  }
  double ml = 1000000.0;
  int mls = -1;
  for (int i = S_PHARYNX0; i <= S_LAST_MOUTH; ++i) {
    double a = X[X_AREA + i - DYN0];
    if (art[i - S_PHARYNX0] == LOWER_LIP && a < ml) { ml = a; mls = i; }
  }
  if (ml < 1.0 && ml < min_teeth) {
    has_l = true;
    cl = Cons{mls, mls, mls, LOWER_LIP, 0.0, 0.0};
    grow(X, art, cl, ml, LOWER_LIP);
    cl.obst = X[X_POS + cl.last + 1 - S_PHARYNX0];
  }
  dipole_targets(X, T, C, teeth, cg);
  if (has_t1) dipole_targets(X, T, C, teeth, ct1);
  if (has_t2) dipole_targets(X, T, C, teeth, ct2);
  if (has_l) dipole_targets(X, T, C, teeth, cl);
}

// Phase A (all lanes): amplitude smoothing of owned dipoles (TdsModel.cpp:1637-1666).
template <int W>
AFS_HD inline void phase_noise_amp(int gl, Lane<W> &R, double *X, const Tables &T) {
  using S = Shape<W>;
  #pragma unroll
  for (int k = 0; k < S::NDP; ++k) {
    int d = gl + k * W;
    if (d >= NDIP) continue;
    double cn = X[X_CUTN + d];
    if (cn != 0.0) R.dcut[k] = cn;  // targeted this step: cutoff was (re)assigned
    double old = R.damp[k];
    double amp = old + T.noise_amp_F * (X[X_TGT + d] - old);
    R.damp[k] = amp;
    if (old >= THR && amp < THR) R.dout[k] = 0.0;
    X[X_ACT + d] = (amp < THR) ? 0.0 : 1.0;
  }
}

// Phase R (lane 0): random inputs of the active sources, in source order (TdsModel.cpp:1690-1696).
AFS_HD inline void phase_noise_rng(double *X, const Tables &T) {
  int32_t *rng = (int32_t *)(X + X_RNG);
  for (int d = 0; d < NDIP; ++d) {
    if (X[X_ACT + d] == 0.0) continue;
    uint32_t acc = 0;
    for (int k = 0; k < 12; ++k) acc += (uint32_t)rng_next(rng);
    double xi = (double)(int32_t)acc;
    xi /= (double)2147483647;
    xi -= 6.0;
    xi /= T.sqrt12;
    X[X_TGT + d] = xi;  // X_TGT is free again: reused for the inputs
  }
}

// Phase F (all lanes): one-pole shaping filter of owned active dipoles (TdsModel.cpp:1672-1707).
template <int W>
AFS_HD inline void phase_noise_filter(int gl, Lane<W> &R, double *X, const Tables &T) {
  using S = Shape<W>;
  #pragma unroll
  for (int k = 0; k < S::NDP; ++k) {
    int d = gl + k * W;
    if (d >= NDIP) continue;
    double smp = 0.0;
    if (X[X_ACT + d] != 0.0) {
      double cut = R.dcut[k];
      double x = (cut == 2000.0) ? T.noise_x_2000 : exp(-2.0 * PI * (cut * T.dt));
      double y = (1.0 - x) * X[X_TGT + d];
      y += x * R.dout[k];
      R.dout[k] = y;
      smp = y * R.damp[k];
    }
    X[X_SMP + d] = smp;
  }
}

// ---------------------------------------------------------------------------
// Phase M: matrix rows (TdsModel.cpp:1785-2039), written as the SPD matrix A = -M, b = -rhs.
// Owner of section s writes row s (its in-current), the edges of section s and, for
// s = 64 / 83, the two radiation rows.
// ---------------------------------------------------------------------------
AFS_HD inline double sec_L(const double *X, const Consts &C, int s) {
  return (s >= DYN0 && s < DYN0 + NDYNS) ? X[X_L + s - DYN0] : C.stat[static_index(s)][ST_L];
}
AFS_HD inline double sec_R1(const double *X, const Consts &C, int s) {
  return (s >= DYN0 && s < DYN0 + NDYNS) ? X[X_R1 + s - DYN0] : C.stat[static_index(s)][ST_R];
}

template <int W>
AFS_HD inline void phase_rows(int gl, Lane<W> &R, double *X, const Tables &T, const Consts &C) {
  using S = Shape<W>;
  const double dt = T.dt;
  const afs_options &opt = T.opt;
#pragma unroll
  for (int j = 0; j < S::NSL; ++j) {
    const int s = slot_section<W>(j, gl);
    if (s < 0) continue;
    const bool dyn = j < S::ND;
    const int i = s;  // current i flows into section s
    const double *ks = C.stat[static_index(s)];
    const double LB = dyn ? X[X_L + s - DYN0] : ks[ST_L];
    const double RB = dyn ? X[X_R0 + s - DYN0] : ((s == S_FOSSA0 && !opt.piriform_fossa) ? T.fossa_R0 : ks[ST_R]);
    const double R1B = dyn ? X[X_R1 + s - DYN0] : ks[ST_R];
    const double AB = dyn ? X[X_AREA + s - DYN0] : T.area[S_LAST_NOSE];  // static: only used by s = 83
    const double EB = X[X_E + s], DB = X[X_D + s];
    const int a = C.topo[i][TP_SRC];
    double LA = 0.0, RA = 0.0, EA = 0.0, DA = 0.0;
    if (a != -1) { LA = sec_L(X, C, a); RA = sec_R1(X, C, a); EA = X[X_E + a]; DA = X[X_D + a]; }
    double LAB = LA + LB, RAB = RA + RB;
    int br = -1;
    if (a != -1) br = (C.topo[a][TP_OUT0] == i) ? C.topo[a][TP_OUT1] : C.topo[a][TP_OUT0];
    double Sx = 0.0;
    if (s >= S_PHARYNX0 && s <= S_LAST_MOUTH) Sx -= X[X_SMP + s - S_PHARYNX0];
    if (s == 0) Sx -= X[X_GP + 1];  // lung pressure source at section 0
    double m, rhs;
    if (br != -1) {
      double uB = R.u[j], uBr = R.ur[j], uD = X[X_U + br], uDr = X[X_UR + br];
      double F = LAB / (dt * TH) + RAB;
      double H = -(1.0 / (dt * TH)) * (LAB * uB + LA * uD) - (TH1 / TH) * (LAB * uBr + LA * uDr) + Sx;
      m = -EB - EA - F;
      rhs = H + DB - DA;
    } else {
      double uu = R.u[j], uur = R.ur[j];
      if (opt.inner_length_corrections && a >= S_PHARYNX0 && s <= S_LAST_MOUTH)
        LAB += junction_l(X[X_AREA + a - DYN0], AB);
      double G = LAB / (dt * TH) + RAB;
      double H = -uur * LAB * (TH1 / TH) - (LAB * uu) / (dt * TH) + Sx;
      m = -EB - G;
      if (a != -1) m -= EA;
      rhs = H + DB;
      if (a != -1) rhs -= DA;
    }
    X[X_DIAG + i] = -m;
    X[X_RHS + i] = -rhs;
    // edges of section s: (in, out0) = -E, (in, out1) = -E, (out0, out1) = E + L/(dt th) + R1
    const int e0 = C.topo[s][TP_E0], e1 = C.topo[s][TP_E1], e2 = C.topo[s][TP_E2];
    if (e0 >= 0) X[X_OFF + e0] = -EB;
    if (e1 >= 0) {
      X[X_OFF + e1] = -EB;
      X[X_OFF + e2] = -(-EB - (LB / (dt * TH) + R1B));
    }
    if (s == S_LAST_MOUTH || s == S_LAST_NOSE) {  // radiation rows (TdsModel.cpp:1841-1911)
      const int rc = C.topo[s][TP_OUT0], lc = C.topo[s][TP_OUT1];
      double uR = X[X_U + rc], uL = X[X_U + lc], uRr = X[X_UR + rc], uLr = X[X_UR + lc];
      R.rad_u[0] = uR; R.rad_u[1] = uL; R.rad_ur[0] = uRr; R.rad_ur[1] = uLr;
      R.rad_un[0] = X[X_UN + rc]; R.rad_un[1] = X[X_UN + lc];
      const double LA2 = LB, RA2 = R1B, Sr = -X[X_SMP + DIP_LIPS];
      {
        double Rrad = T.rrad_num / (9.0 * PI * PI * AB);
        double F = LA2 / (dt * TH) + RA2 + Rrad;
        double H = -(LA2 / (dt * TH)) * (uR + uL) - (LA2 * (TH1 / TH)) * (uRr + uLr) + Sr;
        X[X_DIAG + rc] = -(-EB - F);
        X[X_RHS + rc] = -(H - DB);
      }
      {
        double Lrad = T.lrad_num / (3.0 * PI * sqrt(AB * PI));
        double LAB2 = LA2 + Lrad;
        double G = LAB2 / (dt * TH) + RA2;
        double H = -(1.0 / (dt * TH)) * (LA2 * uR + LAB2 * uL) - (TH1 / TH) * (LA2 * uRr + LAB2 * uLr) + Sr;
        X[X_DIAG + lc] = -(-EB - G);
        X[X_RHS + lc] = -(H - DB);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Solver rounds (chain lanes 0..3).
// ---------------------------------------------------------------------------
AFS_HD inline void solve_forward(int k, int r, double *X, const Consts &C) {
  const SolveStep st = C.step[r][k];
  if (st.c < 0) return;
  double d = X[X_DIAG + st.c];
  double inv = (d < 0.0) ? NAN : 1.0 / d;  // the reference takes sqrt of a negative pivot
  double y = X[X_RHS + st.c];
  if (st.n0 >= 0) {
    double a0 = X[X_OFF + st.e0];
    double f0 = a0 * inv;
    X[X_DIAG + st.n0] -= f0 * a0;
    X[X_RHS + st.n0] -= f0 * y;
    if (st.n1 >= 0) {
      double a1 = X[X_OFF + st.e1];
      double f1 = a1 * inv;
      X[X_DIAG + st.n1] -= f1 * a1;
      X[X_RHS + st.n1] -= f1 * y;
      X[X_OFF + st.e01] -= f0 * a1;
    }
  }
  X[X_DIAG + st.c] = inv;
}

AFS_HD inline void solve_backward(int k, int r, double *X, const Consts &C) {
  const SolveStep st = C.step[r][k];
  if (st.c < 0) return;
  double y = X[X_RHS + st.c];
  if (st.n0 >= 0) y -= X[X_OFF + st.e0] * X[X_U + st.n0];
  if (st.n1 >= 0) y -= X[X_OFF + st.e1] * X[X_U + st.n1];
  X[X_U + st.c] = y * X[X_DIAG + st.c];
}

// ---------------------------------------------------------------------------
// Phase U: updateVariables (TdsModel.cpp:2046-2098).
// ---------------------------------------------------------------------------
template <int W>
AFS_HD inline void phase_update(int gl, Lane<W> &R, double *X, const Tables &T, const Consts &C) {
  using S = Shape<W>;
  const double dt = T.dt, c = T.noise_lp_c;
#pragma unroll
  for (int j = 0; j < S::NSL; ++j) {
    const int s = slot_section<W>(j, gl);
    if (s < 0) continue;
    double alpha, beta;
    if (j < S::ND) { alpha = R.al[j]; beta = R.be[j]; }
    else { alpha = C.stat[static_index(s)][ST_ALPHA]; beta = static_beta<W>(R, j, T, C, s); }  // same values as phase_network
    const double unew = X[X_U + s];
    const double uold = R.u[j];
    R.u[j] = unew;
    R.ur[j] = (unew - uold) / (dt * TH) - (TH1 / TH) * R.ur[j];
    R.un[j] = (1.0 - c) * unew + c * R.un[j];
    X[X_UR + s] = R.ur[j];
    X[X_UN + s] = R.un[j];
    double cin = 0.0;
    cin += unew;
    double cout = 0.0;
    const int o0 = C.topo[s][TP_OUT0], o1 = C.topo[s][TP_OUT1];
    if (o0 != -1) cout += X[X_U + o0];
    if (o1 != -1) cout += X[X_U + o1];
    double net = cin - cout;
    double old = R.p[j];
    double p = X[X_D + s] + X[X_E + s] * net;
    R.p[j] = p;
    double prr = (p - old) / (dt * TH) - R.pr[j] * (TH1 / TH);
    R.pr[j] = prr;
    double ow = R.w[j], owr = R.wr[j];
    double w = prr * alpha + beta;
    R.w[j] = w;
    double wr = (w - ow) / (dt * TH) - owr * (TH1 / TH);
    R.wr[j] = wr;
    R.wr2[j] = (wr - owr) / (dt * TH) - R.wr2[j] * (TH1 / TH);
    if (s >= S_LAST_TRACHEA && s <= S_PHARYNX0) X[X_P4 + s - S_LAST_TRACHEA] = p;
    if (s == S_LAST_MOUTH || s == S_LAST_NOSE) {  // the two radiation currents of this section
      for (int q = 0; q < 2; ++q) {
        const int rc = q == 0 ? o0 : o1;
        double un = X[X_U + rc];
        double ur = (un - R.rad_u[q]) / (dt * TH) - (TH1 / TH) * R.rad_ur[q];
        X[X_UR + rc] = ur;
        X[X_UN + rc] = (1.0 - c) * un + c * R.rad_un[q];
      }
    }
  }
}

// Phase O (lane 0): radiated flow, glottal tone, output filter (TdsModel.cpp:687-705,
// Synthesizer.cpp:614-627).  Returns the audio sample.
AFS_HD inline double phase_output(double *X, const Tables &T) {
  double flow = 0.0;
  flow += X[X_U + 93];
  flow += X[X_U + 94];
  flow += X[X_U + 95];
  flow += X[X_U + 96];
  if (T.opt.radiation_from_skin) flow += iir_run(X + X_TONE, 4, T.tone_a, T.tone_b, X[X_P4 + 3]);
  double op = (flow - X[X_PREVFLOW]) / T.dt;
  X[X_PREVFLOW] = flow;
  double y = iir_run(X + X_OUTF, 8, T.out_a, T.out_b, op);
  double smp = y * 0.004;
  smp = smp / 32767;
  if (!isfinite(smp)) X[X_NONFIN] = 1.0;
  return smp;
}

// ---------------------------------------------------------------------------
// One audio sample.  Xc: execution policy (par / one / lanes / sync).
// ---------------------------------------------------------------------------
template <int W, class Xc>
AFS_HD inline void sample_step(Xc &x, double *X, const Tables &T, const Consts &C, double ratio) {
  x.par([&](int gl, Lane<W> &R) { phase_geometry<W>(gl, R, X, T, ratio); });
  x.sync();
  x.par([&](int gl, Lane<W> &R) { phase_network<W>(gl, R, X, T, C); });
  x.sync();
  if (T.opt.generate_noise_sources) {
    x.one([&](Lane<W> &R) { phase_constrictions<W>(R, X, T, C); });
    x.sync();
    x.par([&](int gl, Lane<W> &R) { phase_noise_amp<W>(gl, R, X, T); });
    x.sync();
    x.one([&](Lane<W> &R) { (void)R; phase_noise_rng(X, T); });
    x.sync();
    x.par([&](int gl, Lane<W> &R) { phase_noise_filter<W>(gl, R, X, T); });
  } else {
    x.par([&](int gl, Lane<W> &R) {
      (void)R;
      for (int d = gl; d < NDIP; d += W) X[X_SMP + d] = 0.0;
    });
  }
  x.sync();
  x.par([&](int gl, Lane<W> &R) { phase_rows<W>(gl, R, X, T, C); });
  x.sync();
  for (int r = 0; r < T.n_rounds; ++r) {
    x.lanes(TREE_CHAINS, [&](int k, Lane<W> &R) { (void)R; solve_forward(k, r, X, C); });
    x.sync();
  }
  for (int r = T.n_rounds - 1; r >= 0; --r) {
    x.lanes(TREE_CHAINS, [&](int k, Lane<W> &R) { (void)R; solve_backward(k, r, X, C); });
    x.sync();
  }
  x.par([&](int gl, Lane<W> &R) { phase_update<W>(gl, R, X, T, C); });
  x.sync();
  x.one([&](Lane<W> &R) { R.sample = phase_output(X, T); });
}

}  // namespace tree
}  // namespace afs
