// tds_lane.hip -- "lane" kernels: one GPU lane owns one utterance.
//
// This is the reference-order path (afs_solver AFS_SOLVER_CHOLESKY): per sample it runs
// exactly the reference's stages -- Tube::interpolate, TriangularGlottis::calcGeometry /
// incTime, TdsModel::prepareTimeStep (with calcNoiseSources), calcMatrix, the
// symmetric-envelope Cholesky and updateVariables, then the output filter
// (Synthesizer.cpp:557-629, TdsModel.cpp:659-711) -- with the reference's operand order, so
// that apart from device exp()/pow() it reproduces the CPU result bit for bit.
//
// Layout: every per-utterance quantity q[k] lives at ws[(OFF_q + k) * bp + u]; consecutive
// lanes hold consecutive utterances, so every access of the time loop is a coalesced 512-B
// wave access.  The whole time loop runs inside the kernel (persistent in time); the kernel
// is compiled with -ffp-contract=off to keep the reference's rounding.
#include <hip/hip_runtime.h>

#include "afs_model.h"
#include "afs_lane.h"

namespace afs {

namespace {

struct Col {
  double *p;
  int64_t s;
  __device__ double &operator[](int i) const { return p[(int64_t)i * s]; }
};

__device__ __forceinline__ double clampA(double a) { return a < AMIN ? AMIN : a; }

struct Lane {
  const Tables &T;
  double *base;
  int64_t bp;
  int32_t *rng;
  bool sor;  // solveEquationsSor instead of solveEquationsCholesky
  __device__ Col q(int off) const { return Col{base + (int64_t)off * bp, bp}; }

  __device__ int32_t rand_next() const {
    int f = rng[31 * bp];
    int r = f - 3;
    if (r < 0) r += 31;
    uint32_t v = (uint32_t)rng[f * bp] + (uint32_t)rng[r * bp];
    rng[f * bp] = (int32_t)v;
    rng[31 * bp] = (f + 1 == 31) ? 0 : f + 1;
    return (int32_t)(v >> 1);
  }
};

// glibc __srandom_r (random_r.c): Schrage LCG fill, then 310 discarded outputs.
// rng[k * bp] holds state word k (k < 31); rng[31 * bp] is the ring index of fptr.
__device__ void seed_rng(int32_t *rng, int64_t bp, uint32_t seed) {
  if (seed == 0) seed = 1;
  int32_t word = (int32_t)seed;
  rng[0] = word;
  for (int i = 1; i < 31; ++i) {
    long hi = word / 127773;
    long lo = word % 127773;
    long nw = 16807 * lo - 2836 * hi;
    if (nw < 0) nw += 2147483647;
    word = (int32_t)nw;
    rng[i * bp] = word;
  }
  int f = 3;
  for (int k = 0; k < 310; ++k) {
    int r = f - 3;
    if (r < 0) r += 31;
    rng[f * bp] = (int32_t)((uint32_t)rng[f * bp] + (uint32_t)rng[r * bp]);
    f = (f + 1 == 31) ? 0 : f + 1;
  }
  rng[31 * bp] = f;
}

// ---------------------------------------------------------------------------
// TriangularGlottis (TriangularGlottis.cpp:154-576).  relx: cur0, cur1, prev0, prev1.
// ---------------------------------------------------------------------------
// TwoMassModel (TwoMassModel.cpp): calcGeometry/getTubeData (:359-440), then incTime
// (:157-349), in the reference's operand order.
__device__ void two_mass_glottis(const double gp[6], const Col &RELX, const Col &P, const Col &AREA,
                                 const Col &LEN, const Col &VOL, double T) {
  double Q = 1.0 + (gp[0] - TM_NAT_F0) / TM_F0_DIV_Q;
  if (Q < 0.05) Q = 0.05;
  const double f = sqrt(Q);
  const double len = TM_REST_LEN * f, th0 = TM_REST_THICK0 / f, th1 = TM_REST_THICK1 / f;
  const double rel[2] = {RELX[0], RELX[1]}, prev[2] = {RELX[2], RELX[3]};
  const double rest[2] = {gp[2], gp[3]};
  {
    double ab[2];
    for (int i = 0; i < 2; ++i) {
      ab[i] = rest[i] + rel[i];
      if (ab[i] < 0.0) ab[i] = 0.0;
    }
    double passive = 2.0 * gp[3];
    if (passive < 0.0) passive = 0.0;
    double chink = passive * TM_CHINK_LEN + gp[4];
    if (chink < 0.0) chink = 0.0;
    const double a0 = clampA(2.0 * len * ab[0] + chink), a1 = clampA(2.0 * len * ab[1] + chink);
    AREA[S_GLOT_LO] = a0; LEN[S_GLOT_LO] = th0; VOL[S_GLOT_LO] = a0 * th0;
    AREA[S_GLOT_UP] = a1; LEN[S_GLOT_UP] = th1; VOL[S_GLOT_UP] = a1 * th1;
  }
  const double pr[4] = {P[S_LAST_TRACHEA], P[S_GLOT_LO], P[S_GLOT_UP], P[S_PHARYNX0]};
  const double critX = 0.5 * TM_CRIT_WIDTH;
  const double ab[2] = {rest[0] + rel[0], rest[1] + rel[1]};
  const double minRel[2] = {critX - rest[0], critX - rest[1]};
  const double m[2] = {TM_MASS0 / Q, TM_MASS1 / Q};
  const double k[2] = {TM_K0 * Q, TM_K1 * Q};
  const double eta[2] = {TM_ETA0, TM_ETA1};
  double ck[2] = {TM_KC0 * Q, TM_KC1 * Q};
  double ceta[2] = {TM_CETA0, TM_CETA1};
  const double kc = TM_KCOUPLE * Q * Q;
  const double df = gp[5];
  double dr[2] = {TM_DAMP0, TM_DAMP1};
  if (ab[0] <= critX) dr[0] += 1.0;
  if (ab[1] <= critX) dr[1] += 1.0;
  const double r[2] = {2.0 * dr[0] * sqrt(m[0] * k[0]) * df * df, 2.0 * dr[1] * sqrt(m[1] * k[1]) * df * df};
  double fo[2];
  if ((ab[0] > TM_CRIT_WIDTH) && (ab[1] > TM_CRIT_WIDTH)) {
    fo[0] = pr[1] * len * th0; fo[1] = pr[2] * len * th1;
  } else if ((ab[0] <= TM_CRIT_WIDTH) && (ab[1] > TM_CRIT_WIDTH)) {
    fo[0] = pr[0] * len * th0; fo[1] = pr[2] * len * th1;
  } else if ((ab[0] > TM_CRIT_WIDTH) && (ab[1] <= TM_CRIT_WIDTH)) {
    fo[0] = pr[1] * len * th0; fo[1] = pr[1] * len * th1;
  } else {
    fo[0] = pr[0] * len * th0; fo[1] = pr[3] * len * th1;
  }
  double nl[2];
  for (int i = 0; i < 2; ++i) {
    if (rel[i] > minRel[i]) { ck[i] = 0.0; ceta[i] = 0.0; }
    const double dx = rel[i] - minRel[i];
    nl[i] = k[i] * eta[i] * rel[i] * rel[i] * rel[i] + ck[i] * ceta[i] * dx * dx * dx;
  }
  const double A = m[0] + r[0] * T + T * T * (k[0] + ck[0]) + kc * T * T;
  const double B = -kc * T * T;
  const double Cq = -kc * T * T;
  const double D = m[1] + r[1] * T + T * T * (k[1] + ck[1]) + kc * T * T;
  const double E = fo[0] * T * T + 2.0 * m[0] * rel[0] - m[0] * prev[0] + r[0] * T * rel[0] +
                   T * T * ck[0] * minRel[0] - nl[0] * T * T;
  const double F = fo[1] * T * T + 2.0 * m[1] * rel[1] - m[1] * prev[1] + r[1] * T * rel[1] +
                   T * T * ck[1] * minRel[1] - nl[1] * T * T;
  double det = A * D - B * Cq;
  if (fabs(det) < 0.000000001) det = 0.000000001;
  RELX[2] = rel[0];
  RELX[3] = rel[1];
  RELX[0] = (E * D - B * F) / det;
  RELX[1] = (A * F - E * Cq) / det;
}

__device__ __forceinline__ double glottis_q(double f0) {
  double q = 1.0 + (f0 - G_NAT_F0) / G_F0_DIV_Q;
  return q < 0.05 ? 0.05 : q;
}

__device__ void glottis_open_close(const double gp[6], double rel0, double rel1, double olen[2],
                                   double clen[2], double ow[2], double cz[2]) {
  double q = glottis_q(gp[0]);
  double cord = G_REST_LEN * sqrt(q);
  double rest[2] = {gp[2], gp[3]};
  double rel[2] = {rel0, rel1};
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

// ---------------------------------------------------------------------------
// One output sample for one utterance (Synthesizer.cpp:557-627).
// ---------------------------------------------------------------------------
enum : int {
  Q_P = 0, Q_PR = Q_P + NS, Q_W = Q_PR + NS, Q_WR = Q_W + NS, Q_WR2 = Q_WR + NS,
  Q_U = Q_WR2 + NS, Q_UR = Q_U + NC, Q_UN = Q_UR + NC,
  Q_DAMP = Q_UN + NC, Q_DOUT = Q_DAMP + NDIP, Q_DCUT = Q_DOUT + NDIP,
  Q_GBF = Q_DCUT + NDIP, Q_TONE = Q_GBF + 1, Q_OUTF = Q_TONE + 8, Q_PREVFLOW = Q_OUTF + 16,
  Q_RELX = Q_PREVFLOW + 1, Q_NONFINITE = Q_RELX + 4,
  Q_TGLOT = Q_NONFINITE + 1, Q_TVEL1 = Q_TGLOT + 8, Q_TVEL2 = Q_TVEL1 + 8,  // option filters
  Q_PERSIST = Q_TVEL2 + 8,
  Q_AREA = Q_PERSIST, Q_LEN = Q_AREA + NS, Q_VOL = Q_LEN + NS, Q_POS = Q_VOL + NS,
  Q_LAT = Q_POS + NS, Q_ART = Q_LAT + NS,
  Q_L = Q_ART + NS, Q_C = Q_L + NS, Q_R0 = Q_C + NS, Q_R1 = Q_R0 + NS, Q_AL = Q_R1 + NS,
  Q_BE = Q_AL + NS, Q_D = Q_BE + NS, Q_E = Q_D + NS,
  Q_DTGT = Q_E + NS, Q_DSMP = Q_DTGT + NDIP, Q_SOL = Q_DSMP + NDIP, Q_FLOW = Q_SOL + NC,
  Q_FDIAG = Q_FLOW + NC, Q_FENV = Q_FDIAG + NC
};

struct Cons { int first, last, narrow, art; double obst, lat; };

__device__ void grow(const Col &AREA, const Col &ART, Cons &c, double amin_, int art) {
  double amax = amin_ + 0.2;
  while (AREA[c.first] < amax && (int)ART[c.first] == art && c.first > S_PHARYNX0) c.first--;
  while (AREA[c.last] < amax && (int)ART[c.last] == art && c.last < S_LAST_MOUTH) c.last++;
  c.first++;
  c.last--;
}

__device__ void tongue_obstacle(const Col &AREA, const Col &POS, const Col &LEN, const Col &LAT,
                                double teeth, Cons &c, double &min_teeth) {
  for (int i = c.first; i <= c.last; ++i)
    if (LAT[i] > c.lat) c.lat = LAT[i];
  double jet = POS[c.last] + LEN[c.last];
  if (teeth - jet < 2.0) {
    c.obst = teeth;
    min_teeth = AREA[c.narrow];
  } else {
    c.obst = POS[c.last + 1] + 0.5 * LEN[c.last + 1];
  }
}

// calcNoiseSources (TdsModel.cpp:1188-1622) + calcNoiseSample (:1630-1708).
__device__ void noise_sources(const Lane &Ln, double teeth, double asp) {
  const Tables &T = Ln.T;
  Col AREA = Ln.q(Q_AREA), ART = Ln.q(Q_ART), POS = Ln.q(Q_POS), LEN = Ln.q(Q_LEN), LAT = Ln.q(Q_LAT);
  Col UN = Ln.q(Q_UN), TGT = Ln.q(Q_DTGT), AMP = Ln.q(Q_DAMP), DOUT = Ln.q(Q_DOUT), CUT = Ln.q(Q_DCUT);
  Col SMP = Ln.q(Q_DSMP);
  for (int i = 0; i < NDIP; ++i) TGT[i] = 0.0;
  Cons cs[4];
  int nc = 1;
  cs[0] = Cons{S_GLOT_LO, S_GLOT_UP, S_GLOT_UP, VOCAL_FOLDS, 1.5, 0.0};
  double min_teeth = 1000000.0, mt = 1000000.0;
  int mts = -1;
  for (int i = S_PHARYNX0; i <= S_LAST_MOUTH; ++i)
    if ((int)ART[i] == TONGUE && AREA[i] < mt) { mt = AREA[i]; mts = i; }
  if (mt < 1.0) {
    Cons &c = cs[nc++];
    c = Cons{mts, mts, mts, TONGUE, 0.0, 0.0};
    grow(AREA, ART, c, mt, TONGUE);
    tongue_obstacle(AREA, POS, LEN, LAT, teeth, c, min_teeth);
  }
  if (cs[nc - 1].art == TONGUE) {
    const Cons pc = cs[nc - 1];
    mt = 1000000.0;
    mts = -1;
    for (int i = S_PHARYNX0; i <= S_LAST_MOUTH; ++i)
      if ((int)ART[i] == TONGUE && AREA[i] < mt && (i < pc.first || i > pc.last)) { mt = AREA[i]; mts = i; }
    if (mt < 1.0) {
      Cons &c = cs[nc++];
      c = Cons{mts, mts, mts, TONGUE, 0.0, 0.0};
      grow(AREA, ART, c, mt, TONGUE);
      if (c.first > pc.last + 1 || c.last < pc.first - 1) tongue_obstacle(AREA, POS, LEN, LAT, teeth, c, min_teeth);
      else nc--;
    }
  }
  double ml = 1000000.0;
  int mls = -1;
  for (int i = S_PHARYNX0; i <= S_LAST_MOUTH; ++i)
    if ((int)ART[i] == LOWER_LIP && AREA[i] < ml) { ml = AREA[i]; mls = i; }
  if (ml < 1.0 && ml < min_teeth) {
    Cons &c = cs[nc++];
    c = Cons{mls, mls, mls, LOWER_LIP, 0.0, 0.0};
    grow(AREA, ART, c, ml, LOWER_LIP);
    c.obst = POS[c.last + 1];
  }
  for (int k = 0; k < nc; ++k) {
    const Cons c = cs[k];
    int ob = -1;
    for (int i = S_PHARYNX0; i <= S_LAST_MOUTH && ob == -1; ++i)
      if (POS[i] <= c.obst && POS[i] + LEN[i] >= c.obst) ob = i;
    if (ob == -1) continue;
    int up = ob - S_PHARYNX0;
    int dn = (ob < S_LAST_MOUTH) ? up + 1 : DIP_LIPS;
    double fdn = (c.obst - POS[ob]) / LEN[ob];
    double fup = 1.0 - fdn;
    double A = (c.narrow >= S_PHARYNX0) ? AREA[c.narrow] : AREA[c.narrow];
    if (A < 0.1) A = 0.1;
    double flow = 0.0;
    int o0 = T.cout0[c.narrow], o1 = T.cout1[c.narrow];
    if (o0 != -1) flow += UN[o0];
    if (o1 != -1) flow += UN[o1];
    if (flow < 0.0) flow = 0.0;
    double v = flow / A;
    double fc = 6000.0, gain = 0.0;
    if (c.art == LOWER_LIP) {
      gain = 2.0e-7;
    } else if (c.art == VOCAL_FOLDS) {
      gain = 0.5e-7 * pow(10.0, asp / 20.0);
    } else {
      double d = sqrt(4.0 * A / PI);
      fc = 0.15 * v / d;
      gain = (fabs(c.obst - teeth) < 0.0001) ? 10.0e-7 : 5.0e-7;
    }
    double full = gain * fabs(v) * v * v * sqrt(A);
    if (c.lat > 0.1) full = 0.0;
    if (fc < 50.0) fc = 50.0;
    if (fc > 2000.0) fc = 2000.0;
    TGT[up] = fup * full; CUT[up] = fc;
    TGT[dn] = fdn * full; CUT[dn] = fc;
  }
  const double F = T.noise_amp_F;
  for (int d = 0; d < NDIP; ++d) {
    double old = AMP[d];
    double amp = old + F * (TGT[d] - old);
    AMP[d] = amp;
    if (old >= 0.001 && amp < 0.001) DOUT[d] = 0.0;
    if (amp < 0.001) { SMP[d] = 0.0; continue; }
    double cut = CUT[d];
    double x = (cut == 2000.0) ? T.noise_x_2000 : exp(-2.0 * PI * (cut * T.dt));
    double a0 = 1.0 - x;
    uint32_t acc = 0;
    for (int k = 0; k < 12; ++k) acc += (uint32_t)Ln.rand_next();
    double xi = (double)(int32_t)acc;
    xi /= (double)2147483647;
    xi -= 6.0;
    xi /= T.sqrt12;
    double y = a0 * xi;
    y += x * DOUT[d];
    DOUT[d] = y;
    SMP[d] = y * amp;
  }
}

__device__ __forceinline__ double junction_l(double A1, double A2) {
  if (A1 < AMIN) A1 = AMIN;
  if (A2 < AMIN) A2 = AMIN;
  double a, b;
  if (A1 > A2) { a = sqrt(A1 / PI); b = sqrt(A2 / PI); }
  else { a = sqrt(A2 / PI); b = sqrt(A1 / PI); }
  double H = 1.0 - b / a;
  return 8.0 * RHO * H / (3.0 * PI * PI * b);
}

// getGlottalEntranceLossCoeffFlucher2011(pressure, d) (TdsModel.cpp:1048-1092)
__device__ double fulcher_kent(double pressure_dPa, double d_cm) {
  double pc = pressure_dPa / 979.7;
  double D = d_cm;
  if (pc < 0.001) pc = 0.001;
  if (D < 0.001) D = 0.001;
  double logD = log10(D);
  double a = pow(10.0, 0.7953 * logD * logD + 1.4741 * logD + 0.6529);
  double b = -0.7427 * logD * logD + -1.6209 * logD + -0.875;
  double k = a * pow(pc, b);
  if (k < 0.6) k = 0.6;
  if (k > 18.0) k = 18.0;
  return k;
}

// solveEquationsSor (TdsModel.cpp:2105-2180) on the negated envelope storage of calcMatrix
// (negating A and b leaves every SOR iterate bit-identical).  Entry (i, j > i) is read from
// row j's envelope: calcMatrix writes the two halves with identical values.
__device__ void sor_solve(const Lane &Ln, const Col &AREA, const Col &FD, const Col &FE, const Col &SOL,
                          const Col &FLOW) {
  const Tables &T = Ln.T;
  uint64_t act0 = ~0ull, act1 = ~0ull;  // isActive bit per current (97 bits)
  auto off = [&](int c) {
    if (c < 0) return;
    if (c < 64) act0 &= ~(1ull << c); else act1 &= ~(1ull << (c - 64));
  };
  for (int i = 0; i < NS; ++i) {
    const double a = is_static_section(i) ? T.area[i] : AREA[i];
    if (a <= 1.01 * AMIN) { off(T.cin[i]); off(T.cout0[i]); off(T.cout1[i]); }
  }
  for (int i = 0; i < NC; ++i) FLOW[i] = 0.0;
  auto m = [&](int i, int j) -> double {
    return j < i ? FE[T.env_off[i] + j - T.env_start[i]] : FE[T.env_off[j] + i - T.env_start[j]];
  };
  int it = 0;
  double res;
  do {
    res = 0.0;
    for (int i = NC - 1; i >= 0; --i) {
      const bool active = i < 64 ? ((act0 >> i) & 1) : ((act1 >> (i - 64)) & 1);
      if (!active) continue;
      double sum = FD[i] * FLOW[i];
      for (int k = T.row_n[i] - 1; k >= 0; --k) {
        const int j = T.row[i][k];
        sum += FLOW[j] * m(i, j);
      }
      const double d = SOL[i] - sum;
      res += d * d;
      FLOW[i] = FLOW[i] + 1.25 * d / FD[i];
    }
    ++it;
  } while (it < 100 && res > 0.1 * 0.1);
}

__device__ double iir_step(const Col &st, int order, const double *a, const double *b, double x) {
  // st[0..order-1] = previous inputs (newest first), st[order..2order-1] = previous outputs.
  double acc = a[0] * x;
  for (int k = 1; k <= order; ++k) {
    acc += a[k] * st[k - 1];
    acc += b[k] * st[order + k - 1];
  }
  for (int k = order - 1; k > 0; --k) { st[k] = st[k - 1]; st[order + k] = st[order + k - 1]; }
  st[0] = x;
  st[order] = acc;
  return acc;
}

__device__ double sample_step(const Lane &Ln, const afs_frame *fl, const afs_frame *fr, double ratio) {
  const Tables &T = Ln.T;
  const afs_options &opt = T.opt;
  Col P = Ln.q(Q_P), PR = Ln.q(Q_PR), W = Ln.q(Q_W), WR = Ln.q(Q_WR), WR2 = Ln.q(Q_WR2);
  Col U = Ln.q(Q_U), UR = Ln.q(Q_UR), UN = Ln.q(Q_UN);
  Col AREA = Ln.q(Q_AREA), LEN = Ln.q(Q_LEN), VOL = Ln.q(Q_VOL), POS = Ln.q(Q_POS);
  Col LAT = Ln.q(Q_LAT), ART = Ln.q(Q_ART);
  Col Lc = Ln.q(Q_L), Cc = Ln.q(Q_C), R0 = Ln.q(Q_R0), R1 = Ln.q(Q_R1), AL = Ln.q(Q_AL), BE = Ln.q(Q_BE);
  Col D = Ln.q(Q_D), E = Ln.q(Q_E), SMP = Ln.q(Q_DSMP);
  Col SOL = Ln.q(Q_SOL), FLOW = Ln.q(Q_FLOW), FD = Ln.q(Q_FDIAG), FE = Ln.q(Q_FENV);
  Col RELX = Ln.q(Q_RELX);
  const double dt = T.dt;
  const double r1 = 1.0 - ratio;

  // Tube::interpolate (Tube.cpp:438-505) -> pharynx/mouth and velum sections.
  double x = 0.0;
  for (int i = 0; i < NPM; ++i) {
    int k = S_PHARYNX0 + i;
    double a = r1 * clampA(fl->area_cm2[i]) + ratio * clampA(fr->area_cm2[i]);
    double l = r1 * fl->length_cm[i] + ratio * fr->length_cm[i];
    double lt = r1 * fl->laterality[i] + ratio * fr->laterality[i];
    POS[k] = x;
    LEN[k] = l;
    a = clampA(a);
    AREA[k] = a;
    VOL[k] = a * l;
    ART[k] = (double)fl->articulator[i];
    LAT[k] = lt;
    x += l;
  }
  const double teeth = r1 * fl->teeth_position_cm + ratio * fr->teeth_position_cm;
  const double open = r1 * clampA(fl->velum_opening_cm2) + ratio * clampA(fr->velum_opening_cm2);
  for (int i = 0; i < 4; ++i) {
    int k = S_NOSE0 + i;
    double a = clampA(open + ((double)(i * i) * (T.nose4_area - open)) / (double)16);
    AREA[k] = a;
    LEN[k] = T.len[k];
    VOL[k] = a * T.len[k];
  }
  // Glottis controls (Synthesizer.cpp:572-575) and calcGeometry (TriangularGlottis.cpp:338-397).
  double gp[6];
  for (int k = 0; k < 6; ++k) gp[k] = r1 * fl->glottis[k] + ratio * fr->glottis[k];
  const double rel0 = RELX[0], rel1 = RELX[1];
  const bool two_mass = opt.glottis_model == AFS_GLOTTIS_TWO_MASS;
  if (two_mass) {
    two_mass_glottis(gp, RELX, P, AREA, LEN, VOL, 1.0 / T.fs);
  } else {
  {
    double chink = gp[4] < 0.0 ? 0.0 : gp[4];
    double f = sqrt(glottis_q(gp[0]));
    double th0 = G_REST_THICK0 / f, th1 = G_REST_THICK1 / f;
    double olen[2], clen[2], ow[2], cz[2];
    glottis_open_close(gp, rel0, rel1, olen, clen, ow, cz);
    double a0 = clampA(olen[0] * ow[0] + chink), a1 = clampA(olen[1] * ow[1] + chink);
    AREA[S_GLOT_LO] = a0; LEN[S_GLOT_LO] = th0; VOL[S_GLOT_LO] = a0 * th0;
    AREA[S_GLOT_UP] = a1; LEN[S_GLOT_UP] = th1; VOL[S_GLOT_UP] = a1 * th1;
  }
  // TriangularGlottis::incTime (TriangularGlottis.cpp:154-330) with the previous pressures.
  {
    const double Tt = 1.0 / T.fs;
    const double pr0 = P[S_LAST_TRACHEA], pr1 = P[S_GLOT_LO], pr2 = P[S_GLOT_UP], pr3 = P[S_PHARYNX0];
    double q = glottis_q(gp[0]);
    double f = sqrt(q);
    double cord = G_REST_LEN * f;
    double th[2] = {G_REST_THICK0 / f, G_REST_THICK1 / f};
    double olen[2], clen[2], ow[2], cz[2];
    glottis_open_close(gp, rel0, rel1, olen, clen, ow, cz);
    double m0 = G_MASS0 / q, m1 = G_MASS1 / q;
    double al0 = clen[0] / cord, al1 = clen[1] / cord;
    double k0 = G_K0 * q, k1 = G_K1 * q, kc0 = G_KC0 * q, kc1 = G_KC1 * q;
    double kcp = G_KCOUPLE * q * q;
    double dr0 = G_DAMP0 + al0 * 1.0, dr1 = G_DAMP1 + al1 * 1.0;
    double rr0 = 2.0 * dr0 * sqrt(m0 * k0), rr1 = 2.0 * dr1 * sqrt(m1 * k1);
    double fo0 = pr1 * olen[0] * th[0];
    double fo1 = pr2 * olen[1] * th[1];
    fo0 += 0.5 * 0.5 * (pr0 + pr1) * G_INLET * cord;
    fo1 += 0.5 * 0.5 * (pr3 + pr2) * G_OUTLET * cord;
    double rs0 = (gp[2] >= 0.0) ? gp[2] * (1.0 - cz[0] / cord) : gp[2];
    double rs1 = (gp[3] >= 0.0) ? gp[3] * (1.0 - cz[1] / cord) : gp[3];
    double A = m0 + rr0 * Tt + Tt * Tt * (k0 + kc0 * al0) + kcp * Tt * Tt;
    double B = -kcp * Tt * Tt;
    double Cq = -kcp * Tt * Tt;
    double Dq = m1 + rr1 * Tt + Tt * Tt * (k1 + kc1 * al1) + kcp * Tt * Tt;
    double Ee = fo0 * Tt * Tt + 2.0 * m0 * rel0 - m0 * RELX[2] + rr0 * Tt * rel0 - Tt * Tt * kc0 * al0 * rs0;
    double Ff = fo1 * Tt * Tt + 2.0 * m1 * rel1 - m1 * RELX[3] + rr1 * Tt * rel1 - Tt * Tt * kc1 * al1 * rs1;
    double det = A * Dq - B * Cq;
    if (fabs(det) < 0.000000001) det = 0.000000001;
    RELX[2] = rel0;
    RELX[3] = rel1;
    RELX[0] = (Ee * Dq - B * Ff) / det;
    RELX[1] = (A * Ff - Ee * Cq) / det;
  }
  }

  // ---- TdsModel::prepareTimeStep (TdsModel.cpp:718-1010) ----
  for (int i = 0; i < NS; ++i) {
    if (is_static_section(i)) {
      Lc[i] = T.L[i]; Cc[i] = T.C[i]; R0[i] = T.R[i]; R1[i] = T.R[i];
      AL[i] = T.alpha[i];
      BE[i] = opt.soft_walls ? T.alpha[i] * (W[i] * T.wc1[i] + WR[i] * T.wc2[i] + WR2[i] * T.Lw[i] * (TH1 / TH)) : 0.0;
      continue;
    }
    double area = AREA[i], len = LEN[i], vol = VOL[i];
    double circ = 2.0 * sqrt(area * PI);
    double a = sqrt(area / PI), b = a;
    double rmin = (i == S_GLOT_LO || i == S_GLOT_UP) ? 0.8 : 1.6;
    if (a < rmin) { a = rmin; b = area / (PI * a); }
    Lc[i] = (RHO * 0.5 * len) / area;
    Cc[i] = vol / (RHO * CSND * CSND);
    double R = ((2.0 * MU * len) * (a * a + b * b)) / (PI * a * a * a * b * b * b);
    R0[i] = R; R1[i] = R;
    double alpha = 0.0, beta = 0.0;
    if (opt.soft_walls && i != S_GLOT_LO && i != S_GLOT_UP) {
      double surf = circ * len;
      if (surf < AMIN) surf = AMIN;
      double Rw = T.Bw[i] / surf, Lw = T.Mw[i] / surf, Cw = surf / T.Kw[i];
      alpha = 1.0 / (Lw / (dt * dt * TH * TH) + Rw / (dt * TH) + 1.0 / Cw);
      beta = alpha * (W[i] * (Lw / (dt * dt * TH * TH) + Rw / (dt * TH)) +
                      WR[i] * (Lw * (TH1 / TH + 1.0) / (dt * TH) + Rw * (TH1 / TH)) +
                      WR2[i] * Lw * (TH1 / TH));
    }
    AL[i] = alpha;
    BE[i] = beta;
  }
  if (opt.turbulence_losses) {
    for (int i = S_PHARYNX0 + 1; i <= S_LAST_MOUTH; ++i) {
      int a = i - 1;
      if (T.cout0[a] != -1 && T.cout1[a] == -1) {
        double u = 0.0;
        u += U[T.cout0[a]];
        double Ai = AREA[i], Aa = AREA[a];
        if ((Ai < Aa && u > 0) || (Ai > Aa && u < 0)) {
          R1[a] = R1[a] - u * 0.5 * RHO / (Aa * Aa);
          R0[i] = R0[i] + u * 0.5 * RHO / (Ai * Ai);
        }
      }
    }
  }
  if (!opt.piriform_fossa) R0[S_FOSSA0] = T.fossa_R0;
  {
    Col GBF = Ln.q(Q_GBF);
    double kent = 1.0;  // glottal entrance loss (TdsModel.cpp:898-911, 1019-1092)
    if (opt.glottis_loss == AFS_ENTRANCE_LOSS_VAN_DEN_BERG) {
      kent = 1.375;
    } else if (opt.glottis_loss == AFS_ENTRANCE_LOSS_VARIABLE) {
      double tp = P[S_LAST_TRACHEA] - P[S_PHARYNX0];
      double ftp = iir_step(Ln.q(Q_TGLOT), 4, T.tglot_a, T.tglot_b, tp);
      kent = fulcher_kent(ftp, AREA[S_GLOT_LO] / 1.25);
    }
    double sa = T.area[S_LAST_TRACHEA], ta = AREA[S_GLOT_LO];
    double u = 0.0;
    u += U[S_GLOT_LO];
    if (u > 0) R0[S_GLOT_LO] = R0[S_GLOT_LO] + kent * 0.5 * RHO * fabs(u) * (1.0 / (ta * ta) - 1.0 / (sa * sa));
    sa = AREA[S_GLOT_LO];
    ta = AREA[S_GLOT_UP];
    double bt = (ta < opt.flow_separation_area_ratio * sa) ? 1.0 : 0.0;
    double g = 0.8 * GBF[0] + (1.0 - 0.8) * bt;
    GBF[0] = g;
    u = 0.0;
    u += U[S_GLOT_UP];
    if (u > 0) R1[S_GLOT_LO] = R1[S_GLOT_LO] + g * fabs(u) * 0.5 * RHO * (1.0 / (ta * ta) - 1.0 / (sa * sa));
  }
  if (opt.generate_noise_sources) noise_sources(Ln, teeth, two_mass ? GLOTTIS_DEFAULT_ASPIRATION_DB : gp[5]);
  else for (int d = 0; d < NDIP; ++d) SMP[d] = 0.0;
  double tvflow = 0.0;  // transvelar coupling (TdsModel.cpp:966-980)
  if (opt.transvelar_coupling)
    tvflow = iir_step(Ln.q(Q_TVEL1), 4, T.tone_a, T.tone_b, P[S_MOUTH0 + 2]) +
             iir_step(Ln.q(Q_TVEL2), 4, T.tvel2_a, T.tone_b, P[S_NOSE0 + 2]);
  for (int i = 0; i < NS; ++i) {
    double d = is_static_section(i) ? T.E[i] : dt * TH / (Cc[i] + AL[i]);
    double src = 0.0;
    if (i == S_NOSE0 + 2) src += tvflow;
    E[i] = d;
    D[i] = P[i] + T.dtTH1 * PR[i] - d * (BE[i] - src);
  }

  // ---- calcMatrix (TdsModel.cpp:1785-2039) into the negated envelope storage ----
  const double lips = SMP[DIP_LIPS];
  const double p_amp = gp[1];
  for (int i = 0; i < NC; ++i) {
    const int es = T.env_start[i], eo = T.env_off[i];
    for (int j = es; j < i; ++j) FE[eo + j - es] = -(0.0);
  }
  auto put = [&](int i, int j, double m) {
    if (j == i) FD[i] = -m;
    else if (j < i) FE[T.env_off[i] + j - T.env_start[i]] = -m;
  };
  for (int i = 0; i < NC; ++i) {
    const int sa_ = T.src[i], tb_ = T.tgt[i];
    double rhs;
    if (tb_ == -1) {
      const int rc = T.cout0[sa_], lc = T.cout1[sa_];
      double uR = U[rc], uL = U[lc], uRr = UR[rc], uLr = UR[lc];
      double LA = Lc[sa_], RA = R1[sa_];
      double S = -lips;
      double Arad = (sa_ == S_LAST_MOUTH) ? AREA[sa_] : T.area[sa_];
      double F, G, H;
      if (i == rc) {
        double Rrad = T.rrad_num / (9.0 * PI * PI * Arad);
        F = LA / (dt * TH) + RA + Rrad;
        G = LA / (dt * TH) + RA;
        H = -(LA / (dt * TH)) * (uR + uL) - (LA * (TH1 / TH)) * (uRr + uLr) + S;
      } else {
        double Lrad = T.lrad_num / (3.0 * PI * sqrt(Arad * PI));
        double LAB = LA + Lrad;
        F = LA / (dt * TH) + RA;
        G = LAB / (dt * TH) + RA;
        H = -(1.0 / (dt * TH)) * (LA * uR + LAB * uL) - (TH1 / TH) * (LA * uRr + LAB * uLr) + S;
      }
      if (T.cin[sa_] != -1) put(i, T.cin[sa_], E[sa_]);
      put(i, rc, -E[sa_] - F);
      put(i, lc, -E[sa_] - G);
      rhs = H - D[sa_];
    } else {
      double LB = Lc[tb_], RB = R0[tb_];
      double LA = 0.0, RA = 0.0;
      if (sa_ != -1) { LA = Lc[sa_]; RA = R1[sa_]; }
      double LAB = LA + LB, RAB = RA + RB;
      int br = -1;
      if (sa_ != -1) br = (T.cout0[sa_] == i) ? T.cout1[sa_] : T.cout0[sa_];
      double S = 0.0;
      S -= (tb_ >= S_PHARYNX0 && tb_ <= S_LAST_MOUTH) ? SMP[tb_ - S_PHARYNX0] : 0.0;
      if (tb_ == 0) S -= p_amp;
      if (br != -1) {
        double uB = U[i], uBr = UR[i], uD = U[br], uDr = UR[br];
        double F = LAB / (dt * TH) + RAB;
        double G = LA / (dt * TH) + RA;
        double H = -(1.0 / (dt * TH)) * (LAB * uB + LA * uD) - (TH1 / TH) * (LAB * uBr + LA * uDr) + S;
        put(i, br, -E[sa_] - G);
        if (T.cin[sa_] != -1) put(i, T.cin[sa_], E[sa_]);
        put(i, i, -E[tb_] - E[sa_] - F);
        if (T.cout0[tb_] != -1) put(i, T.cout0[tb_], E[tb_]);
        if (T.cout1[tb_] != -1) put(i, T.cout1[tb_], E[tb_]);
        rhs = H + D[tb_] - D[sa_];
      } else {
        double uu = U[i], uur = UR[i];
        if (opt.inner_length_corrections && sa_ >= S_PHARYNX0 && tb_ <= S_LAST_MOUTH)
          LAB += junction_l(AREA[sa_], AREA[tb_]);
        double G = LAB / (dt * TH) + RAB;
        double H = -uur * LAB * (TH1 / TH) - (LAB * uu) / (dt * TH) + S;
        if (sa_ != -1 && T.cin[sa_] != -1) put(i, T.cin[sa_], E[sa_]);
        double m = -E[tb_] - G;
        if (sa_ != -1) m -= E[sa_];
        put(i, i, m);
        if (T.cout0[tb_] != -1) put(i, T.cout0[tb_], E[tb_]);
        if (T.cout1[tb_] != -1) put(i, T.cout1[tb_], E[tb_]);
        rhs = H + D[tb_];
        if (sa_ != -1) rhs -= D[sa_];
      }
    }
    SOL[i] = -rhs;
  }

  if (Ln.sor) {
    sor_solve(Ln, AREA, FD, FE, SOL, FLOW);
  } else {
  // ---- solveEquationsCholesky (TdsModel.cpp:2259-2313) ----
  for (int k = 0; k < NC; ++k) {
    const int esk = T.env_start[k], eok = T.env_off[k];
    double dk = FD[k];
    for (int j = esk; j < k; ++j) {
      double f = FE[eok + j - esk];
      dk -= f * f;
    }
    dk = sqrt(dk);
    FD[k] = dk;
    for (int q = 0; q < T.col_n[k]; ++q) {
      const int i = T.col[k][q];
      const int esi = T.env_start[i], eoi = T.env_off[i];
      double fik = FE[eoi + k - esi];
      for (int j = esk; j < k; ++j) {
        double fij = (j >= esi) ? FE[eoi + j - esi] : 0.0;
        fik -= fij * FE[eok + j - esk];
      }
      FE[eoi + k - esi] = fik / dk;
    }
  }
  for (int k = 0; k < NC; ++k) {
    const int esk = T.env_start[k], eok = T.env_off[k];
    double y = SOL[k];
    for (int j = esk; j < k; ++j) y -= FE[eok + j - esk] * SOL[j];
    SOL[k] = y / FD[k];
  }
  for (int k = NC - 1; k >= 0; --k) {
    double y = SOL[k];
    for (int q = 0; q < T.col_n[k]; ++q) {
      const int i = T.col[k][q];
      y -= FE[T.env_off[i] + k - T.env_start[i]] * FLOW[i];
    }
    SOL[k] = y;
    FLOW[k] = y / FD[k];
  }
  }

  // ---- updateVariables (TdsModel.cpp:2046-2098) ----
  const double c = T.noise_lp_c;
  for (int i = 0; i < NC; ++i) {
    double old = U[i];
    double u = FLOW[i];
    U[i] = u;
    UR[i] = (u - old) / (dt * TH) - (TH1 / TH) * UR[i];
    UN[i] = (1.0 - c) * u + c * UN[i];
  }
  for (int i = 0; i < NS; ++i) {
    double cin = 0.0;
    if (T.cin[i] != -1) cin += U[T.cin[i]];
    double cout = 0.0;
    if (T.cout0[i] != -1) cout += U[T.cout0[i]];
    if (T.cout1[i] != -1) cout += U[T.cout1[i]];
    double net = cin - cout;
    double old = P[i];
    double p = D[i] + E[i] * net;
    P[i] = p;
    double prr = (p - old) / (dt * TH) - PR[i] * (TH1 / TH);
    PR[i] = prr;
    double ow = W[i], owr = WR[i];
    double w = prr * AL[i] + BE[i];
    W[i] = w;
    double wr = (w - ow) / (dt * TH) - owr * (TH1 / TH);
    WR[i] = wr;
    WR2[i] = (wr - owr) / (dt * TH) - WR2[i] * (TH1 / TH);
  }

  // radiated flow (TdsModel.cpp:687-705)
  double flow = 0.0;
  flow += U[93];
  flow += U[94];
  flow += U[95];
  flow += U[96];
  if (opt.radiation_from_skin) flow += iir_step(Ln.q(Q_TONE), 4, T.tone_a, T.tone_b, P[S_PHARYNX0]);
  // output stage (Synthesizer.cpp:614-627)
  Col PF = Ln.q(Q_PREVFLOW);
  double op = (flow - PF[0]) / dt;
  PF[0] = flow;
  double y = iir_step(Ln.q(Q_OUTF), 8, T.out_a, T.out_b, op);
  double smp = y * 0.004;
  return smp / 32767;
}

}  // namespace

// Reset the persistent state of utterances [0, B) and seed their generators (seeds == nullptr:
// utterance u is seeded u + 1, afs.h).
__global__ void lane_reset_kernel(double *ws, int32_t *rng, int64_t bp, int B, const uint32_t *seeds) {
  int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= B) return;
  for (int k = 0; k < Q_PERSIST; ++k) ws[(int64_t)k * bp + u] = 0.0;
  for (int d = 0; d < NDIP; ++d) ws[(int64_t)(Q_DCUT + d) * bp + u] = 3000.0;
  seed_rng(rng + u, bp, seeds ? seeds[u] : (uint32_t)u + 1u);
}

// Time loop over frame transitions k in [k_begin, k_end): pair (frames[k-1], frames[k]).
__global__ void __launch_bounds__(64) lane_synth_kernel(LaneArgs a) {
  int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= a.B) return;
  const Tables &T = *a.tab;
  Lane L{T, a.ws + u, a.bp, a.rng + u, a.sor != 0};
  const afs_frame *fu = a.frames + (int64_t)(a.frame_row ? a.frame_row[u] : u) * a.frame_stride;
  double *o = a.out + (int64_t)u * a.out_stride;
  Col NF = L.q(Q_NONFINITE);
  double bad = NF[0];
  int64_t t = 0;
  for (int k = a.k_begin; k < a.k_end; ++k) {
    const afs_frame *fl = fu + (k - 1);
    const afs_frame *fr = fu + k;
    for (int i = 0; i < a.hop; ++i) {
      double ratio = (double)i / (double)a.hop;
      double s = sample_step(L, fl, fr, ratio);
      if (!isfinite(s)) bad = 1.0;
      o[t++] = s;
    }
  }
  NF[0] = bad;
}

__global__ void lane_nonfinite_kernel(const double *ws, int64_t bp, int B, int32_t *count, uint8_t *flags) {
  int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= B) return;
  const bool nf = ws[(int64_t)Q_NONFINITE * bp + u] != 0.0;
  if (flags) flags[u] = nf ? 1 : 0;
  if (nf) atomicAdd(count, 1);
}

int64_t lane_ws_rows(const Tables &t) { return (int64_t)Q_FENV + t.env_total; }
int64_t lane_persist_rows() { return Q_PERSIST; }

}  // namespace afs

namespace afs {

hipError_t launch_lane_reset(double *ws, int32_t *rng, int64_t bp, int B, const uint32_t *seeds, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(lane_reset_kernel, dim3((B + 63) / 64), dim3(64), 0, st, ws, rng, bp, B, seeds);
  return hipGetLastError();
}

hipError_t launch_lane_synth(const LaneArgs &a, hipStream_t st) {
  if (a.B <= 0 || a.k_end <= a.k_begin) return hipSuccess;
  hipLaunchKernelGGL(lane_synth_kernel, dim3((a.B + 63) / 64), dim3(64), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_lane_nonfinite(const double *ws, int64_t bp, int B, int32_t *count, uint8_t *flags, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(lane_nonfinite_kernel, dim3((B + 63) / 64), dim3(64), 0, st, ws, bp, B, count, flags);
  return hipGetLastError();
}

}  // namespace afs
