/*
 * afs_oracle.c -- CPU restatement of the reference hot path (batch of 1).
 *
 * TEST INFRASTRUCTURE ONLY (see afs_oracle.h).  This file is the checker that the
 * HIP product is compared with; the product never links or calls it.
 *
 * The arithmetic below keeps the reference's operand order and association so the
 * result is bit-identical to the reference compiled with the same flags (gcc -O2,
 * x86-64, no FMA contraction).  Every function names the reference lines it follows.
 * Structure (flat arrays per quantity, explicit topology tables) is our own.
 */
#include "afs_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

_Static_assert(sizeof(ao_frame) == 1072, "ao_frame must match afs_frame");

/* ---------------------------------------------------------------------------
 * Section / current numbering (Tube.h:53-82, TdsModel.h:37).
 * ------------------------------------------------------------------------- */
enum {
  NS = 93, NC = 97,
  S_TRACHEA0 = 0, S_LAST_TRACHEA = 22, S_GLOT_LO = 23, S_GLOT_UP = 24,
  S_PHARYNX0 = 25, S_LAST_PHARYNX = 40, S_MOUTH0 = 41, S_LAST_MOUTH = 64,
  S_NOSE0 = 65, S_LAST_NOSE = 83, S_FOSSA0 = 84, S_LAST_FOSSA = 88,
  S_SINUS0 = 89, S_LAST_SINUS = 92,
  ENV_MAX = 57, COL_MAX = 10
};
enum { ART_VOCAL_FOLDS = 0, ART_TONGUE = 1, ART_LOWER_INCISORS = 2, ART_LOWER_LIP = 3, ART_OTHER = 4 };

/* Physical constants, Constants.h:8-16; TdsModel.cpp:15-22; Tube.cpp:8-16. */
static const double RHO = 1.14e-3;
static const double CSND = 3.5e4;
static const double MU = 1.86e-4;
static const double TH = 0.515;
static const double TH1 = 1.0 - 0.515;
static const double AMIN = 0.1e-2;
static const double NOISE_LP_HZ = 500.0;

/* ---------------------------------------------------------------------------
 * IIR filter (IirFilter.cpp:17-65, 137-150, 235-243, 286-432).
 * ------------------------------------------------------------------------- */
typedef struct iir {
  double a[33], b[33];
  int order, pos;
  double xin[64], yout[64];
} iir;

static void iir_clear(iir *f) {
  memset(f->a, 0, sizeof f->a);
  memset(f->b, 0, sizeof f->b);
  f->b[0] = 1.0;
  f->order = 0;
}
static void iir_reset(iir *f) {
  memset(f->xin, 0, sizeof f->xin);
  memset(f->yout, 0, sizeof f->yout);
  f->pos = 0;
}
/* IirFilter::getOutputSample, IirFilter.cpp:47-65 */
static double iir_run(iir *f, double x) {
  f->xin[f->pos & 63] = x;
  double acc = f->a[0] * x;
  for (int k = 1; k <= f->order; ++k) {
    acc += f->a[k] * f->xin[(f->pos - k) & 63];
    acc += f->b[k] * f->yout[(f->pos - k) & 63];
  }
  f->yout[f->pos & 63] = acc;
  f->pos++;
  return acc;
}

/* IirFilter::createChebyshev, IirFilter.cpp:286-432 (0.5 % ripple). */
static void chebyshev_design(double ratio, int hp, int poles, double *a, double *b, int *order) {
  double ta[33], tb[33];
  if (poles & 1) poles++;
  if (poles > 32) poles = 32;
  *order = poles;
  for (int i = 0; i <= 32; ++i) { a[i] = 0.0; b[i] = 0.0; }
  a[2] = 1.0;
  b[2] = 1.0;
  for (int p = 1; p <= poles / 2; ++p) {
    double re = -cos(M_PI / (2.0 * poles) + (M_PI * (p - 1)) / (double)poles);
    double im = sin(M_PI / (2.0 * poles) + (M_PI * (p - 1)) / (double)poles);
    {
      double tmp = 100.0 / (100.0 - 0.5);
      double es = sqrt(tmp * tmp - 1.0);
      double vx = (1.0 / (double)poles) * log((1.0 / es) + sqrt((1.0 / (es * es)) + 1));
      double kx = (1.0 / (double)poles) * log((1.0 / es) + sqrt((1.0 / (es * es)) - 1));
      kx = 0.5 * (exp(kx) + exp(-kx));
      re = re * (0.5 * (exp(vx) - exp(-vx))) / kx;
      im = im * (0.5 * (exp(vx) + exp(-vx))) / kx;
    }
    double t = 2.0 * tan(0.5);
    double w = 2.0 * M_PI * ratio;
    double m = re * re + im * im;
    double d = 4.0 - 4.0 * re * t + m * t * t;
    double x0 = (t * t) / d, x1 = (2.0 * t * t) / d, x2 = (t * t) / d;
    double y1 = (8.0 - 2.0 * m * t * t) / d;
    double y2 = (-4.0 - 4.0 * re * t - m * t * t) / d;
    double k = hp ? -cos(0.5 * w + 0.5) / cos(0.5 * w - 0.5) : sin(0.5 - 0.5 * w) / sin(0.5 + 0.5 * w);
    d = 1.0 + y1 * k - y2 * k * k;
    double a0 = (x0 - x1 * k + x2 * k * k) / d;
    double a1 = (-2.0 * x0 * k + x1 + x1 * k * k - 2.0 * x2 * k) / d;
    double a2 = (x0 * k * k - x1 * k + x2) / d;
    double b1 = (2.0 * k + y1 + y1 * k * k - 2.0 * y2 * k) / d;
    double b2 = (-(k * k) - y1 * k + y2) / d;
    if (hp) { a1 = -a1; b1 = -b1; }
    memcpy(ta, a, sizeof ta);
    memcpy(tb, b, sizeof tb);
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
  double gain = sa / (1.0 - sb);
  for (int i = 0; i <= 30; ++i) a[i] /= gain;
}

int ao_chebyshev(double cutoff_ratio, int highpass, int poles, double *a, double *b) {
  double ta[33], tb[33];
  int order;
  chebyshev_design(cutoff_ratio, highpass, poles, ta, tb, &order);
  for (int i = 0; i <= order; ++i) { a[i] = ta[i]; b[i] = tb[i]; }
  return order;
}

/* ---------------------------------------------------------------------------
 * glibc random_r TYPE_3 (x_n = x_{n-31} + x_{n-3}, output x_n >> 1).
 * glibc 2.35 stdlib/random_r.c: __srandom_r and __random_r.
 * fptr and rptr always stay 3 apart, so one ring index suffices.
 * ------------------------------------------------------------------------- */
void ao_rng_seed(ao_rng *g, uint32_t seed) {
  if (seed == 0) seed = 1;
  int32_t word = (int32_t)seed;
  g->r[0] = word;
  for (int i = 1; i < 31; ++i) {
    long hi = word / 127773;
    long lo = word % 127773;
    long nw = 16807 * lo - 2836 * hi;
    if (nw < 0) nw += 2147483647;
    word = (int32_t)nw;
    g->r[i] = word;
  }
  g->f = 3;
  for (int k = 0; k < 310; ++k) (void)ao_rng_next(g);
}

int32_t ao_rng_next(ao_rng *g) {
  int f = g->f;
  int r = f - 3;
  if (r < 0) r += 31;
  uint32_t v = (uint32_t)g->r[f] + (uint32_t)g->r[r];
  g->r[f] = (int32_t)v;
  g->f = (f + 1 == 31) ? 0 : f + 1;
  return (int32_t)(v >> 1);
}

/* ---------------------------------------------------------------------------
 * Static network topology (TdsModel::initModel, TdsModel.cpp:67-292).
 * ------------------------------------------------------------------------- */
typedef struct topo {
  int src[NC], tgt[NC];
  int cin[NS], cout0[NS], cout1[NS];
  int env_n[NC], env[NC][ENV_MAX];
  int col_n[NC], col[NC][COL_MAX];
  int row_n[NC], row[NC][16];  /* filledRowIndex (TdsModel.cpp:340-357): ascending, <= 16 */
} topo;

static const int SINUS_COUPLE[4] = {8, 9, 11, 12}; /* Tube.cpp:35-38 */

static void topo_build(topo *t) {
  for (int i = 0; i < NS; ++i) { t->src[i] = i - 1; t->tgt[i] = i; }
  t->src[S_TRACHEA0] = -1;
  t->src[S_NOSE0] = S_LAST_PHARYNX;
  t->src[S_FOSSA0] = S_PHARYNX0 + 3;
  for (int i = 0; i < 4; ++i) t->src[S_SINUS0 + i] = S_NOSE0 + SINUS_COUPLE[i];
  t->src[93] = S_LAST_MOUTH; t->tgt[93] = -1;
  t->src[94] = S_LAST_MOUTH; t->tgt[94] = -1;
  t->src[95] = S_LAST_NOSE;  t->tgt[95] = -1;
  t->src[96] = S_LAST_NOSE;  t->tgt[96] = -1;
  for (int s = 0; s < NS; ++s) { t->cin[s] = -1; t->cout0[s] = -1; t->cout1[s] = -1; }
  for (int c = 0; c < NC; ++c) {
    if (t->src[c] != -1) {
      int s = t->src[c];
      if (t->cout0[s] == -1) t->cout0[s] = c; else t->cout1[s] = c;
    }
    if (t->tgt[c] != -1) t->cin[t->tgt[c]] = c;
  }
  /* Pattern of the coefficient matrix, then the symmetric-envelope index lists. */
  static unsigned char nz[NC][NC];
  memset(nz, 0, sizeof nz);
  for (int c = 0; c < NC; ++c) {
    int sides[2] = {t->src[c], t->tgt[c]};
    for (int q = 0; q < 2; ++q) {
      int s = sides[q];
      if (s == -1) continue;
      if (t->cin[s] != -1) nz[c][t->cin[s]] = 1;
      if (t->cout0[s] != -1) nz[c][t->cout0[s]] = 1;
      if (t->cout1[s] != -1) nz[c][t->cout1[s]] = 1;
    }
    t->row_n[c] = 0;
    for (int j = 0; j < NC; ++j)
      if (nz[c][j] && j != c && t->row_n[c] < 16) t->row[c][t->row_n[c]++] = j;
    t->env_n[c] = 0;
    int inside = 0;
    for (int j = 0; j < c; ++j) {
      if (nz[c][j] || inside) {
        inside = 1;
        nz[c][j] = 1;
        t->env[c][t->env_n[c]++] = j;
      }
    }
  }
  for (int j = 0; j < NC; ++j) {
    t->col_n[j] = 0;
    for (int i = j + 1; i < NC; ++i)
      if (nz[i][j]) t->col[j][t->col_n[j]++] = i;
  }
}

/* ---------------------------------------------------------------------------
 * Per-utterance synthesizer state.
 * ------------------------------------------------------------------------- */
typedef struct noise_src {
  double target, amp, cutoff, sample;
  double xin[8], yout[8];
} noise_src;

struct ao_synth {
  topo T;
  ao_options opt;
  double fs, dt;
  ao_rng rng;
  long rng_calls;

  /* Synthesizer::tube (the interpolated tube), Synthesizer.h:272 */
  double area[NS], len[NS], vol[NS], Mw[NS], Bw[NS], Kw[NS], pos[NS], lat[NS];
  int art[NS];
  double teeth, aspiration_db;

  int latched;
  ao_frame prev;

  /* TriangularGlottis state + control values (TriangularGlottis.h:107-112) */
  double relx[2][4];
  int gpos;
  double gp[6];

  /* TdsModel dynamic state (TdsModel.h:150-201) */
  double p[NS], pr[NS], w[NS], wr[NS], wr2[NS];
  double L[NS], C[NS], R0[NS], R1[NS], Ssrc[NS], alpha[NS], beta[NS], D[NS], E[NS];
  double u[NC], ur[NC], un[NC];
  noise_src dip[NS];
  noise_src lips;
  double gbf;          /* glottalBernoulliFactor */
  double p_amp;        /* pressureSourceAmp at section 0 */
  double teeth_tds, asp_tds;
  int position;
  iir tone;            /* glottalToneFilter */
  iir tglot;           /* transglottalPressureFilter (VARIABLE_ENTRANCE_LOSS) */
  iir tvel1, tvel2;    /* transvelarCouplingFilter1/2 */
  iir outf;            /* Synthesizer::outputPressureFilter */
  double flow_ring[256];
  double sol[NC], flowv[NC];
  int sor_iterations;
  double fac[NC][NC];
  double mat[NC][NC];
};

void ao_default_options(ao_options *o) {
  o->turbulence_losses = 1;
  o->soft_walls = 1;
  o->generate_noise_sources = 1;
  o->radiation_from_skin = 1;
  o->piriform_fossa = 0;
  o->inner_length_corrections = 1;
  o->transvelar_coupling = 0;
  o->glottis_loss = 0;
  o->solver = 0;
  o->glottis_model = 0;
  o->flow_separation_area_ratio = 1.0;
}

/* getGlottalEntranceLossCoeffFlucher2011(pressure, d), TdsModel.cpp:1048-1092. */
double ao_fulcher_kent(double pressure_dPa, double d_cm) {
  double pc = pressure_dPa / 979.7;
  double D = d_cm;
  if (pc < 0.001) pc = 0.001;
  if (D < 0.001) D = 0.001;
  double logD = log10(D);
  double a = pow(10, 0.7953 * logD * logD + 1.4741 * logD + 0.6529);
  double b = -0.7427 * logD * logD + -1.6209 * logD + -0.875;
  double k = a * pow(pc, b);
  if (k < 0.6) k = 0.6;
  if (k > 18.0) k = 18.0;
  return k;
}

/* Static parts of the tube: Tube.cpp:79-260 (trachea, nose, sinuses, fossa) and
 * Tube.cpp:267-314 (dynamic defaults, whose wall data persist). */
static void tube_init(ao_synth *s) {
  static const double NOSE_A[19] = {1.63, 2.07, 2.72, 3.59, 4.24, 3.26, 3.04, 3.04, 2.72, 2.5,
                                     2.39, 2.39, 1.85, 0.76, 1.41, 1.74, 1.30, 1.74, 0.76};
  static const double SIN_V[4] = {11.3, 6.8, 33.0, 6.2};
  static const double NECK_L[4] = {0.3, 0.3, 0.45, 1.0};
  static const double NECK_A[4] = {0.185, 0.185, 0.145, 0.11};
  for (int i = 0; i < NS; ++i) {
    s->Mw[i] = 2.1; s->Bw[i] = 800.0; s->Kw[i] = 84500.0;
    s->art[i] = ART_OTHER; s->lat[i] = 0.0; s->pos[i] = 0.0;
  }
  for (int i = 0; i <= S_LAST_TRACHEA; ++i) {
    s->area[i] = (i == 0) ? 4.0 : (i == 1) ? 3.0 : 2.5;
    s->len[i] = 23.0 / (double)23;
    s->vol[i] = s->area[i] * s->len[i];
    s->Mw[i] = 0.25; s->Bw[i] = 1000.0;
  }
  for (int i = 0; i < 2; ++i) {
    int k = S_GLOT_LO + i;
    s->area[k] = 0.1; s->len[k] = 0.3; s->vol[k] = s->area[k] * s->len[k];
    s->art[k] = ART_VOCAL_FOLDS;
  }
  for (int i = 0; i < 40; ++i) {
    int k = S_PHARYNX0 + i;
    s->area[k] = 4.0; s->len[k] = 16.0 / (double)40; s->vol[k] = s->area[k] * s->len[k];
  }
  double lf = 11.4 / 11.4;
  for (int i = 0; i < 19; ++i) {
    int k = S_NOSE0 + i;
    s->area[k] = NOSE_A[i];
    s->len[k] = lf * 0.6;
    s->vol[k] = s->area[k] * s->len[k];
  }
  for (int i = 0; i < 4; ++i) {
    int k = S_SINUS0 + i;
    s->area[k] = NECK_A[i]; s->len[k] = NECK_L[i]; s->vol[k] = SIN_V[i];
    s->Mw[k] = 0.0; s->Bw[k] = 6500.0;
  }
  double amax = 2.0 * 2.0 / 3.0, sl = 3.0 / (double)5;
  for (int i = 0; i < 5; ++i) {
    int k = S_FOSSA0 + i;
    s->area[k] = amax * (1.0 - (i + 0.5) / (double)5);
    s->len[k] = sl;
    s->vol[k] = s->area[k] * s->len[k];
  }
  s->teeth = 15.0;
  s->aspiration_db = -40.0;
}

static double clamp_amin(double a) { return a < AMIN ? AMIN : a; }

/* Tube::interpolate + setPharynxMouthGeometry + setVelumOpening (Tube.cpp:323-349,
 * 402-416, 438-505).  Frame areas/openings are the stored (clamped) values of the
 * caller's Tube (Tube.cpp:337, 413). */
static void tube_interpolate(ao_synth *s, const ao_frame *fl, const ao_frame *fr, double ratio) {
  double r1 = 1.0 - ratio;
  double x = 0.0;
  for (int i = 0; i < 40; ++i) {
    int k = S_PHARYNX0 + i;
    double a = r1 * clamp_amin(fl->area_cm2[i]) + ratio * clamp_amin(fr->area_cm2[i]);
    double l = r1 * fl->length_cm[i] + ratio * fr->length_cm[i];
    double lt = r1 * fl->laterality[i] + ratio * fr->laterality[i];
    s->pos[k] = x;
    s->len[k] = l;
    s->area[k] = clamp_amin(a);
    s->vol[k] = s->area[k] * l;
    s->art[k] = fl->articulator[i];
    s->lat[k] = lt;
    x += l;
  }
  s->teeth = r1 * fl->teeth_position_cm + ratio * fr->teeth_position_cm;
  double open = r1 * clamp_amin(fl->velum_opening_cm2) + ratio * clamp_amin(fr->velum_opening_cm2);
  double target = s->area[S_NOSE0 + 4];
  for (int i = 0; i < 4; ++i) {
    int k = S_NOSE0 + i;
    s->area[k] = clamp_amin(open + ((double)(i * i) * (target - open)) / (double)16);
    s->vol[k] = s->area[k] * s->len[k];
  }
}

/* ---------------------------------------------------------------------------
 * TriangularGlottis, TriangularGlottis.cpp (static params :38-56).
 * ------------------------------------------------------------------------- */
static const double G_REST_LEN = 1.3, G_REST_THICK0 = 0.24, G_REST_THICK1 = 0.06;
static const double G_MASS0 = 0.12, G_MASS1 = 0.03, G_DAMP0 = 0.1, G_DAMP1 = 0.6;
static const double G_K0 = 80000.0, G_K1 = 8000.0, G_KC0 = 240000.0, G_KC1 = 24000.0;
static const double G_KCOUPLE = 25000.0, G_INLET = 0.05, G_OUTLET = 0.01;
static const double G_NAT_F0 = 129.0, G_F0_DIV_Q = 125.51;

/* getTensionParameter, :438-455 */
static double glottis_q(double f0) {
  double dq = G_F0_DIV_Q;
  if (dq < 0.000001) dq = 0.000001;
  double q = 1.0 + (f0 - G_NAT_F0) / dq;
  return q < 0.05 ? 0.05 : q;
}

/* getOpenCloseDimensions, :474-576 */
static void glottis_open_close(const ao_synth *s, double olen[2], double clen[2], double ow[2], double cz[2]) {
  double q = glottis_q(s->gp[0]);
  double f = sqrt(q);
  double cord = G_REST_LEN * f;
  double rest[2] = {s->gp[2], s->gp[3]};
  double rel[2] = {s->relx[0][s->gpos & 3], s->relx[1][s->gpos & 3]};
  double back[2] = {rest[0] + rel[0], rest[1] + rel[1]};
  double front[2];
  for (int i = 0; i < 2; ++i) front[i] = (rest[i] < 0.0) ? back[i] : rel[i];
  for (int i = 0; i < 2; ++i) {
    olen[i] = 0.0; ow[i] = 0.0; clen[i] = cord; cz[i] = 0.5 * cord;
    if (back[i] > 0.0 && front[i] > 0.0) {
      olen[i] = cord; ow[i] = back[i] + front[i]; clen[i] = 0.0; cz[i] = 0.0;
    } else if (back[i] <= 0.0 && front[i] <= 0.0) {
      olen[i] = 0.0; ow[i] = 0.0; clen[i] = cord; cz[i] = 0.5 * cord;
    } else {
      if (fabs(rest[i]) < 0.000000001) rest[i] = 0.000000001;
      double apex = cord * (1.0 + rel[i] / rest[i]);
      if (apex >= 0.0 && apex <= cord) {
        if (back[i] > 0.0) {
          olen[i] = apex; ow[i] = back[i]; clen[i] = cord - apex; cz[i] = 0.5 * (apex + cord);
        } else {
          olen[i] = cord - apex; ow[i] = front[i]; clen[i] = apex; cz[i] = 0.5 * apex;
        }
      }
    }
  }
}

/* calcGeometry + getTubeData, :338-411 (contact area is a display-only value). */
static void glottis_geometry(const ao_synth *s, double thick[2], double area[2]) {
  double chink = s->gp[4];
  if (chink < 0.0) chink = 0.0;
  double q = glottis_q(s->gp[0]);
  double f = sqrt(q);
  thick[0] = G_REST_THICK0 / f;
  thick[1] = G_REST_THICK1 / f;
  double olen[2], clen[2], ow[2], cz[2];
  glottis_open_close(s, olen, clen, ow, cz);
  area[0] = olen[0] * ow[0] + chink;
  area[1] = olen[1] * ow[1] + chink;
}

/* incTime, :154-330 */
static void glottis_step(ao_synth *s, double T, const double pr[4]) {
  double q = glottis_q(s->gp[0]);
  double rel[2] = {s->relx[0][s->gpos & 3], s->relx[1][s->gpos & 3]};
  double rest[2] = {s->gp[2], s->gp[3]};
  double prev[2] = {s->relx[0][(s->gpos - 1) & 3], s->relx[1][(s->gpos - 1) & 3]};
  double f = sqrt(q);
  double cord = G_REST_LEN * f;
  double th[2] = {G_REST_THICK0 / f, G_REST_THICK1 / f};
  double olen[2], clen[2], ow[2], cz[2];
  glottis_open_close(s, olen, clen, ow, cz);
  double m[2] = {G_MASS0 / q, G_MASS1 / q};
  double al[2] = {clen[0] / cord, clen[1] / cord};
  double k[2] = {G_K0 * q, G_K1 * q};
  double kc[2] = {G_KC0 * q, G_KC1 * q};
  double kcp = G_KCOUPLE * q * q;
  double dr[2] = {G_DAMP0 + al[0] * 1.0, G_DAMP1 + al[1] * 1.0};
  double r[2] = {2.0 * dr[0] * sqrt(m[0] * k[0]), 2.0 * dr[1] * sqrt(m[1] * k[1])};
  double fo[2];
  fo[0] = pr[1] * olen[0] * th[0];
  fo[1] = pr[2] * olen[1] * th[1];
  fo[0] += 0.5 * 0.5 * (pr[0] + pr[1]) * G_INLET * cord;
  fo[1] += 0.5 * 0.5 * (pr[3] + pr[2]) * G_OUTLET * cord;
  double rs[2];
  for (int i = 0; i < 2; ++i) rs[i] = (rest[i] >= 0.0) ? rest[i] * (1.0 - cz[i] / cord) : rest[i];
  double A = m[0] + r[0] * T + T * T * (k[0] + kc[0] * al[0]) + kcp * T * T;
  double B = -kcp * T * T;
  double Cc = -kcp * T * T;
  double Dd = m[1] + r[1] * T + T * T * (k[1] + kc[1] * al[1]) + kcp * T * T;
  double Ee = fo[0] * T * T + 2.0 * m[0] * rel[0] - m[0] * prev[0] + r[0] * T * rel[0] -
              T * T * kc[0] * al[0] * rs[0];
  double Ff = fo[1] * T * T + 2.0 * m[1] * rel[1] - m[1] * prev[1] + r[1] * T * rel[1] -
              T * T * kc[1] * al[1] * rs[1];
  double det = A * Dd - B * Cc;
  if (fabs(det) < 0.000000001) det = 0.000000001;
  s->relx[0][(s->gpos + 1) & 3] = (Ee * Dd - B * Ff) / det;
  s->relx[1][(s->gpos + 1) & 3] = (A * Ff - Ee * Cc) / det;
  s->gpos++;
}

/* ---------------------------------------------------------------------------
 * TwoMassModel (TwoMassModel.cpp, static parameters :36-58, control parameters :17-24): the classical two-mass model
 * with cubic springs; control parameters f0, lung pressure, rest displacements, extra
 * arytenoid area, damping factor.  Part of the reference's sources but not of its
 * executable (CMakeLists.txt:9); selected here with ao_options.glottis_model = 1.
 * ------------------------------------------------------------------------- */
static const double TM_REST_LEN = 1.3, TM_REST_THICK0 = 0.25, TM_REST_THICK1 = 0.05;
static const double TM_MASS0 = 0.125, TM_MASS1 = 0.025, TM_DAMP0 = 0.1, TM_DAMP1 = 0.6;
static const double TM_K0 = 80000.0, TM_K1 = 8000.0, TM_ETA0 = 100.0, TM_ETA1 = 100.0;
static const double TM_KC0 = 240000.0, TM_KC1 = 24000.0, TM_CETA0 = 500.0, TM_CETA1 = 500.0;
static const double TM_KCOUPLE = 25000.0, TM_CRIT_WIDTH = 0.0, TM_NAT_F0 = 158.0, TM_F0_DIV_Q = 100.0;
static const double TM_CHINK_LEN = 0.2;

/* getTensionParameter, :467-485 */
static double tm_q(double f0) {
  double dq = TM_F0_DIV_Q;
  if (dq < 0.000001) dq = 0.000001;
  double q = 1.0 + (f0 - TM_NAT_F0) / dq;
  return q < 0.05 ? 0.05 : q;
}

/* getLengthAndThickness, :491-497 */
static void tm_len_thick(double q, double *len, double th[2]) {
  double f = sqrt(q);
  *len = TM_REST_LEN * f;
  th[0] = TM_REST_THICK0 / f;
  th[1] = TM_REST_THICK1 / f;
}

/* calcGeometry + getTubeData, :359-440 */
static void tm_geometry(const ao_synth *s, double thick[2], double area[2]) {
  double rest[2] = {s->gp[2], s->gp[3]};
  double rel[2] = {s->relx[0][s->gpos & 3], s->relx[1][s->gpos & 3]};
  double ab[2];
  for (int i = 0; i < 2; ++i) {
    ab[i] = rest[i] + rel[i];
    if (ab[i] < 0.0) ab[i] = 0.0;
  }
  double passive = 2.0 * s->gp[3];
  if (passive < 0.0) passive = 0.0;
  double chink = passive * TM_CHINK_LEN + s->gp[4];
  if (chink < 0.0) chink = 0.0;
  double len;
  tm_len_thick(tm_q(s->gp[0]), &len, thick);
  area[0] = 2.0 * len * ab[0] + chink;
  area[1] = 2.0 * len * ab[1] + chink;
}

/* incTime, :157-349 */
static void tm_step(ao_synth *s, double T, const double pr[4]) {
  double Q = tm_q(s->gp[0]);
  double critX = 0.5 * TM_CRIT_WIDTH;
  double rel[2] = {s->relx[0][s->gpos & 3], s->relx[1][s->gpos & 3]};
  double rest[2] = {s->gp[2], s->gp[3]};
  double ab[2] = {rest[0] + rel[0], rest[1] + rel[1]};
  double minRel[2] = {critX - rest[0], critX - rest[1]};
  double prev[2] = {s->relx[0][(s->gpos - 1) & 3], s->relx[1][(s->gpos - 1) & 3]};
  double len, th[2];
  tm_len_thick(Q, &len, th);
  double m[2] = {TM_MASS0 / Q, TM_MASS1 / Q};
  double k[2] = {TM_K0 * Q, TM_K1 * Q};
  double eta[2] = {TM_ETA0, TM_ETA1};
  double ck[2] = {TM_KC0 * Q, TM_KC1 * Q};
  double ceta[2] = {TM_CETA0, TM_CETA1};
  double kc = TM_KCOUPLE * Q * Q;
  double df = s->gp[5];
  double dr[2] = {TM_DAMP0, TM_DAMP1};
  if (ab[0] <= critX) dr[0] += 1.0;
  if (ab[1] <= critX) dr[1] += 1.0;
  double r[2];
  r[0] = 2.0 * dr[0] * sqrt(m[0] * k[0]) * df * df;
  r[1] = 2.0 * dr[1] * sqrt(m[1] * k[1]) * df * df;
  double fo[2];
  if ((ab[0] > TM_CRIT_WIDTH) && (ab[1] > TM_CRIT_WIDTH)) {
    fo[0] = pr[1] * len * th[0];
    fo[1] = pr[2] * len * th[1];
  } else if ((ab[0] <= TM_CRIT_WIDTH) && (ab[1] > TM_CRIT_WIDTH)) {
    fo[0] = pr[0] * len * th[0];
    fo[1] = pr[2] * len * th[1];
  } else if ((ab[0] > TM_CRIT_WIDTH) && (ab[1] <= TM_CRIT_WIDTH)) {
    fo[0] = pr[1] * len * th[0];
    fo[1] = pr[1] * len * th[1];
  } else {
    fo[0] = pr[0] * len * th[0];
    fo[1] = pr[3] * len * th[1];
  }
  double nl[2];
  for (int i = 0; i < 2; ++i) {
    if (rel[i] > minRel[i]) { ck[i] = 0.0; ceta[i] = 0.0; }
    double dx = rel[i] - minRel[i];
    nl[i] = k[i] * eta[i] * rel[i] * rel[i] * rel[i] + ck[i] * ceta[i] * dx * dx * dx;
  }
  double A = m[0] + r[0] * T + T * T * (k[0] + ck[0]) + kc * T * T;
  double B = -kc * T * T;
  double Cc = -kc * T * T;
  double Dd = m[1] + r[1] * T + T * T * (k[1] + ck[1]) + kc * T * T;
  double Ee = fo[0] * T * T + 2.0 * m[0] * rel[0] - m[0] * prev[0] + r[0] * T * rel[0] +
              T * T * ck[0] * minRel[0] - nl[0] * T * T;
  double Ff = fo[1] * T * T + 2.0 * m[1] * rel[1] - m[1] * prev[1] + r[1] * T * rel[1] +
              T * T * ck[1] * minRel[1] - nl[1] * T * T;
  double det = A * Dd - B * Cc;
  if (fabs(det) < 0.000000001) det = 0.000000001;
  s->relx[0][(s->gpos + 1) & 3] = (Ee * Dd - B * Ff) / det;
  s->relx[1][(s->gpos + 1) & 3] = (A * Ff - Ee * Cc) / det;
  s->gpos++;
}

/* ---------------------------------------------------------------------------
 * TdsModel time step.
 * ------------------------------------------------------------------------- */
static double cur_in(const ao_synth *s, int sec) {
  double f = 0.0;
  if (s->T.cin[sec] != -1) f += s->u[s->T.cin[sec]];
  return f;
}
static double cur_out(const ao_synth *s, int sec) {
  double f = 0.0;
  if (s->T.cout0[sec] != -1) f += s->u[s->T.cout0[sec]];
  if (s->T.cout1[sec] != -1) f += s->u[s->T.cout1[sec]];
  return f;
}

/* calcNoiseSample, TdsModel.cpp:1630-1708 (sources are always first order here:
 * calcNoiseSources sets isFirstOrder = true, :1596/:1600). */
static void noise_sample(ao_synth *s, noise_src *n, double thr) {
  const double F = 1.0 - exp(-2.0 * M_PI * 40.0 * s->dt);
  double old = n->amp;
  n->amp += F * (n->target - n->amp);
  if (old >= thr && n->amp < thr) {
    memset(n->xin, 0, sizeof n->xin);
    memset(n->yout, 0, sizeof n->yout);
  }
  if (n->amp < thr) { n->sample = 0.0; return; }
  double xr = exp(-2.0 * M_PI * (n->cutoff * s->dt));
  double fa0 = 1.0 - xr, fa1 = 0.0, fb1 = xr;
  int32_t acc = 0;
  for (int k = 0; k < 12; ++k) acc = (int32_t)((uint32_t)acc + (uint32_t)ao_rng_next(&s->rng));
  s->rng_calls += 12;
  double x = (double)acc;
  x /= (double)2147483647;
  x -= 6.0;
  x /= sqrt(12.0);
  int ps = s->position;
  n->xin[ps & 7] = x;
  double acc2 = fa0 * x;
  acc2 += fa1 * n->xin[(ps - 1) & 7];
  acc2 += fb1 * n->yout[(ps - 1) & 7];
  n->yout[ps & 7] = acc2;
  n->sample = acc2 * n->amp;
}

typedef struct cons { int first, last, narrow, art; double obst, lat; } cons;

/* Grow a constriction around its narrowest section (TdsModel.cpp:1258-1269). */
static void grow(const ao_synth *s, cons *c, double amin_, int art) {
  double amax = amin_ + 0.2;
  while (s->area[c->first] < amax && s->art[c->first] == art && c->first > S_PHARYNX0) c->first--;
  while (s->area[c->last] < amax && s->art[c->last] == art && c->last < S_LAST_MOUTH) c->last++;
  c->first++;
  c->last--;
}

/* Tongue constriction obstacle (TdsModel.cpp:1271-1300). */
static void tongue_obstacle(const ao_synth *s, cons *c, double *min_for_teeth) {
  for (int i = c->first; i <= c->last; ++i)
    if (s->lat[i] > c->lat) c->lat = s->lat[i];
  double jet = s->pos[c->last] + s->len[c->last];
  if (s->teeth_tds - jet < 2.0) {
    c->obst = s->teeth_tds;
    *min_for_teeth = s->area[c->narrow];
  } else {
    c->obst = s->pos[c->last + 1] + 0.5 * s->len[c->last + 1];
  }
}

/* calcNoiseSources, TdsModel.cpp:1188-1622. */
static void noise_sources(ao_synth *s) {
  cons cs[4];
  int nc = 0;
  for (int i = 0; i < NS; ++i) s->dip[i].target = 0.0;
  s->lips.target = 0.0;

  cs[0].first = S_GLOT_LO; cs[0].last = S_GLOT_UP; cs[0].narrow = S_GLOT_UP;
  cs[0].obst = 1.5; cs[0].art = ART_VOCAL_FOLDS; cs[0].lat = 0.0;
  nc = 1;

  double min_teeth = 1000000.0;
  double mt = 1000000.0;
  int mts = -1;
  for (int i = S_PHARYNX0; i <= S_LAST_MOUTH; ++i)
    if (s->art[i] == ART_TONGUE && s->area[i] < mt) { mt = s->area[i]; mts = i; }
  if (mt < 1.0) {
    cons *c = &cs[nc++];
    c->art = ART_TONGUE; c->lat = 0.0; c->narrow = mts; c->first = mts; c->last = mts;
    grow(s, c, mt, ART_TONGUE);
    tongue_obstacle(s, c, &min_teeth);
  }
  if (nc > 0 && cs[nc - 1].art == ART_TONGUE) {
    cons *pc = &cs[nc - 1];
    mt = 1000000.0;
    mts = -1;
    for (int i = S_PHARYNX0; i <= S_LAST_MOUTH; ++i)
      if (s->art[i] == ART_TONGUE && s->area[i] < mt && (i < pc->first || i > pc->last)) {
        mt = s->area[i];
        mts = i;
      }
    if (mt < 1.0) {
      cons *c = &cs[nc++];
      c->art = ART_TONGUE; c->lat = 0.0; c->narrow = mts; c->first = mts; c->last = mts;
      grow(s, c, mt, ART_TONGUE);
      if (c->first > pc->last + 1 || c->last < pc->first - 1) tongue_obstacle(s, c, &min_teeth);
      else nc--;
    }
  }
  double ml = 1000000.0;
  int mls = -1;
  for (int i = S_PHARYNX0; i <= S_LAST_MOUTH; ++i)
    if (s->art[i] == ART_LOWER_LIP && s->area[i] < ml) { ml = s->area[i]; mls = i; }
  if (ml < 1.0 && ml < min_teeth) {
    cons *c = &cs[nc++];
    c->art = ART_LOWER_LIP; c->lat = 0.0; c->narrow = mls; c->first = mls; c->last = mls;
    grow(s, c, ml, ART_LOWER_LIP);
    c->obst = s->pos[c->last + 1];
  }

  for (int k = 0; k < nc; ++k) {
    cons *c = &cs[k];
    int ob = -1;
    for (int i = S_PHARYNX0; i <= S_LAST_MOUTH && ob == -1; ++i)
      if (s->pos[i] <= c->obst && s->pos[i] + s->len[i] >= c->obst) ob = i;
    if (ob == -1) continue;
    noise_src *up = &s->dip[ob];
    noise_src *dn = (ob < S_LAST_MOUTH) ? &s->dip[ob + 1] : &s->lips;
    double fdn = (c->obst - s->pos[ob]) / s->len[ob];
    double fup = 1.0 - fdn;
    double A = s->area[c->narrow];
    if (A < 0.1) A = 0.1;
    double flow = 0.0;
    if (s->T.cout0[c->narrow] != -1) flow += s->un[s->T.cout0[c->narrow]];
    if (s->T.cout1[c->narrow] != -1) flow += s->un[s->T.cout1[c->narrow]];
    if (flow < 0.0) flow = 0.0;
    double v = flow / A;
    double fc = 6000.0, gain = 0.0;
    if (c->art == ART_LOWER_LIP) {
      gain = 2.0e-7; fc = 6000.0;
    } else if (c->art == ART_VOCAL_FOLDS) {
      gain = 0.5e-7 * pow(10.0, s->asp_tds / 20.0); fc = 6000.0;
    } else {
      double d = sqrt(4.0 * A / M_PI);
      fc = 0.15 * v / d;
      gain = (fabs(c->obst - s->teeth_tds) < 0.0001) ? 10.0e-7 : 5.0e-7;
    }
    double full = gain * fabs(v) * v * v * sqrt(A);
    if (c->lat > 0.1) full = 0.0;
    if (fc < 50.0) fc = 50.0;
    if (fc > 2000.0) fc = 2000.0;
    up->target = fup * full; up->cutoff = fc;
    dn->target = fdn * full; dn->cutoff = fc;
  }
  /* Monopole sources of sections 25..64 never receive a target (only dipoles do),
   * so their amplitude stays exactly 0 and they never draw random numbers
   * (TdsModel.cpp:1615-1620); only the dipoles are run here, in the same order. */
  for (int i = S_PHARYNX0; i <= S_LAST_MOUTH; ++i) noise_sample(s, &s->dip[i], 0.001);
  noise_sample(s, &s->lips, 0.001);
}

/* prepareTimeStep, TdsModel.cpp:718-1010. */
static void tds_prepare(ao_synth *s) {
  const double dt = s->dt;
  for (int i = 0; i < NS; ++i) {
    if (s->area[i] < AMIN) s->area[i] = AMIN;
    s->Ssrc[i] = 0.0;
    double circ = 2.0 * sqrt(s->area[i] * M_PI);
    if (i >= S_SINUS0 && i <= S_LAST_SINUS) {
      s->L[i] = RHO * (s->len[i] / s->area[i]);
      s->C[i] = s->vol[i] / (RHO * CSND * CSND);
      s->R0[i] = (8.0 * MU * M_PI * s->len[i]) / (s->area[i] * s->area[i]);
      s->R1[i] = s->R0[i];
    } else {
      double a = sqrt(s->area[i] / M_PI), b = a;
      double rmin = (i == S_GLOT_LO || i == S_GLOT_UP) ? 0.8 : 1.6;
      if (a < rmin) { a = rmin; b = s->area[i] / (M_PI * a); }
      s->L[i] = (RHO * 0.5 * s->len[i]) / s->area[i];
      s->C[i] = s->vol[i] / (RHO * CSND * CSND);
      s->R0[i] = ((2.0 * MU * s->len[i]) * (a * a + b * b)) / (M_PI * a * a * a * b * b * b);
      s->R1[i] = s->R0[i];
    }
    s->alpha[i] = 0.0;
    s->beta[i] = 0.0;
    if (s->opt.soft_walls && i != S_GLOT_LO && i != S_GLOT_UP) {
      double surf;
      if (i >= S_SINUS0 && i <= S_LAST_SINUS)
        surf = 4.0 * M_PI * pow((3.0 * s->vol[i]) / (4.0 * M_PI), 2.0 / 3.0);
      else
        surf = circ * s->len[i];
      if (surf < AMIN) surf = AMIN;
      double Rw = s->Bw[i] / surf, Lw = s->Mw[i] / surf, Cw = surf / s->Kw[i];
      s->alpha[i] = 1.0 / (Lw / (dt * dt * TH * TH) + Rw / (dt * TH) + 1.0 / Cw);
      s->beta[i] = s->alpha[i] * (s->w[i] * (Lw / (dt * dt * TH * TH) + Rw / (dt * TH)) +
                                  s->wr[i] * (Lw * (TH1 / TH + 1.0) / (dt * TH) + Rw * (TH1 / TH)) +
                                  s->wr2[i] * Lw * (TH1 / TH));
    }
  }
  if (s->opt.turbulence_losses) {
    for (int i = S_PHARYNX0 + 1; i <= S_LAST_MOUTH; ++i) {
      int a = i - 1;
      if (s->T.cout0[a] != -1 && s->T.cout1[a] == -1) {
        double u = cur_out(s, a);
        if ((s->area[i] < s->area[a] && u > 0) || (s->area[i] > s->area[a] && u < 0)) {
          s->R1[a] -= u * 0.5 * RHO / (s->area[a] * s->area[a]);
          s->R0[i] += u * 0.5 * RHO / (s->area[i] * s->area[i]);
        }
      }
    }
  }
  if (!s->opt.piriform_fossa)
    s->R0[S_FOSSA0] = 8.0 * MU * s->len[S_FOSSA0] * M_PI / (AMIN * AMIN);

  /* glottal entrance loss, TdsModel.cpp:898-911 (+ :1019-1039 for the variable option) */
  double kent = 1.0;
  if (s->opt.glottis_loss == 1) kent = 1.375;
  else if (s->opt.glottis_loss == 2) {
    double tp = s->p[S_LAST_TRACHEA] - s->p[S_PHARYNX0];
    double ftp = iir_run(&s->tglot, tp);
    kent = ao_fulcher_kent(ftp, s->area[S_GLOT_LO] / 1.25);
  }
  double sa = s->area[S_LAST_TRACHEA], ta = s->area[S_GLOT_LO];
  double u = cur_in(s, S_GLOT_LO);
  if (u > 0) s->R0[S_GLOT_LO] += kent * 0.5 * RHO * fabs(u) * (1.0 / (ta * ta) - 1.0 / (sa * sa));
  sa = s->area[S_GLOT_LO];
  ta = s->area[S_GLOT_UP];
  double bt = 0.0;
  if (ta < s->opt.flow_separation_area_ratio * sa) bt = 1.0;
  s->gbf = 0.8 * s->gbf + (1.0 - 0.8) * bt;
  u = cur_out(s, S_GLOT_LO);
  if (u > 0) s->R1[S_GLOT_LO] += s->gbf * fabs(u) * 0.5 * RHO * (1.0 / (ta * ta) - 1.0 / (sa * sa));

  if (s->opt.generate_noise_sources) noise_sources(s);

  /* transvelar coupling, TdsModel.cpp:966-980 */
  double tvflow = 0.0;
  if (s->opt.transvelar_coupling)
    tvflow = iir_run(&s->tvel1, s->p[S_MOUTH0 + 2]) + iir_run(&s->tvel2, s->p[S_NOSE0 + 2]);

  for (int i = 0; i < NS; ++i) {
    double src = 0.0; /* monopole sample (never active); flow source disabled */
    if (i == S_NOSE0 + 2) src += tvflow;
    double d = dt * TH / (s->C[i] + s->alpha[i]);
    s->E[i] = d;
    s->D[i] = s->p[i] + dt * TH1 * s->pr[i] - d * (s->beta[i] - src);
  }
}

/* getJunctionInductance, TdsModel.cpp:1745-1778. */
static double junction_l(double A1, double A2) {
  if (A1 < AMIN) A1 = AMIN;
  if (A2 < AMIN) A2 = AMIN;
  double a, b;
  if (A1 > A2) { a = sqrt(A1 / M_PI); b = sqrt(A2 / M_PI); }
  else { a = sqrt(A2 / M_PI); b = sqrt(A1 / M_PI); }
  double H = 1.0 - b / a;
  return 8.0 * RHO * H / (3.0 * M_PI * M_PI * b);
}

/* calcMatrix, TdsModel.cpp:1785-2039, written straight into the negated storage
 * used by solveEquationsCholesky (:2239-2253). */
static void tds_matrix(ao_synth *s, double M[NC][NC], double *rhs) {
  const double dt = s->dt;
  for (int i = 0; i < NC; ++i) rhs[i] = 0.0;
  for (int i = 0; i < NC; ++i) {
    int sa_ = s->T.src[i], tb_ = s->T.tgt[i];
    if (tb_ == -1) {
      int rc = s->T.cout0[sa_], lc = s->T.cout1[sa_];
      double uR = s->u[rc], uL = s->u[lc], uRr = s->ur[rc], uLr = s->ur[lc];
      double LA = s->L[sa_], RA = s->R1[sa_];
      double S = -s->lips.sample;
      double Arad = s->area[sa_];
      double F, G, H;
      if (i == rc) {
        double Rrad = (128 * RHO * CSND) / (9.0 * M_PI * M_PI * Arad);
        F = LA / (dt * TH) + RA + Rrad;
        G = LA / (dt * TH) + RA;
        H = -(LA / (dt * TH)) * (uR + uL) - (LA * (TH1 / TH)) * (uRr + uLr) + S;
      } else {
        double Lrad = (8.0 * RHO) / (3.0 * M_PI * sqrt(Arad * M_PI));
        double LAB = LA + Lrad;
        F = LA / (dt * TH) + RA;
        G = LAB / (dt * TH) + RA;
        H = -(1.0 / (dt * TH)) * (LA * uR + LAB * uL) - (TH1 / TH) * (LA * uRr + LAB * uLr) + S;
      }
      if (s->T.cin[sa_] != -1) M[i][s->T.cin[sa_]] = s->E[sa_];
      M[i][rc] = -s->E[sa_] - F;
      M[i][lc] = -s->E[sa_] - G;
      rhs[i] = H - s->D[sa_];
      continue;
    }
    double LB = s->L[tb_], RB = s->R0[tb_];
    double LA = 0.0, RA = 0.0;
    if (sa_ != -1) { LA = s->L[sa_]; RA = s->R1[sa_]; }
    double LAB = LA + LB, RAB = RA + RB;
    int br = -1;
    if (sa_ != -1) br = (s->T.cout0[sa_] == i) ? s->T.cout1[sa_] : s->T.cout0[sa_];
    double S = s->Ssrc[tb_];
    S -= s->dip[tb_].sample;
    if (tb_ == 0) S -= s->p_amp;
    if (br != -1) {
      double uB = s->u[i], uBr = s->ur[i], uD = s->u[br], uDr = s->ur[br];
      double F = LAB / (dt * TH) + RAB;
      double G = LA / (dt * TH) + RA;
      double H = -(1.0 / (dt * TH)) * (LAB * uB + LA * uD) - (TH1 / TH) * (LAB * uBr + LA * uDr) + S;
      M[i][br] = -s->E[sa_] - G;
      if (s->T.cin[sa_] != -1) M[i][s->T.cin[sa_]] = s->E[sa_];
      M[i][i] = -s->E[tb_] - s->E[sa_] - F;
      if (s->T.cout0[tb_] != -1) M[i][s->T.cout0[tb_]] = s->E[tb_];
      if (s->T.cout1[tb_] != -1) M[i][s->T.cout1[tb_]] = s->E[tb_];
      rhs[i] = H + s->D[tb_] - s->D[sa_];
    } else {
      double uu = s->u[i], uur = s->ur[i];
      if (s->opt.inner_length_corrections && sa_ >= S_PHARYNX0 && tb_ <= S_LAST_MOUTH)
        LAB += junction_l(s->area[sa_], s->area[tb_]);
      double G = LAB / (dt * TH) + RAB;
      double H = -uur * LAB * (TH1 / TH) - (LAB * uu) / (dt * TH) + S;
      if (sa_ != -1 && s->T.cin[sa_] != -1) M[i][s->T.cin[sa_]] = s->E[sa_];
      M[i][i] = -s->E[tb_] - G;
      if (sa_ != -1) M[i][i] -= s->E[sa_];
      if (s->T.cout0[tb_] != -1) M[i][s->T.cout0[tb_]] = s->E[tb_];
      if (s->T.cout1[tb_] != -1) M[i][s->T.cout1[tb_]] = s->E[tb_];
      rhs[i] = H + s->D[tb_];
      if (sa_ != -1) rhs[i] -= s->D[sa_];
    }
  }
}

/* solveEquationsCholesky, TdsModel.cpp:2231-2314 (symmetric-envelope Cholesky). */
static void tds_cholesky(ao_synth *s, double M[NC][NC]) {
  const topo *t = &s->T;
  double (*F)[NC] = s->fac;
  double *y = s->sol;
  for (int i = 0; i < NC; ++i) {
    F[i][i] = -M[i][i];
    for (int v = 0; v < t->env_n[i]; ++v) F[i][t->env[i][v]] = -M[i][t->env[i][v]];
  }
  for (int i = 0; i < NC; ++i) y[i] = -y[i];
  for (int k = 0; k < NC; ++k) {
    for (int v = 0; v < t->env_n[k]; ++v) {
      int j = t->env[k][v];
      F[k][k] -= F[k][j] * F[k][j];
    }
    F[k][k] = sqrt(F[k][k]);
    for (int q = 0; q < t->col_n[k]; ++q) {
      int i = t->col[k][q];
      for (int v = 0; v < t->env_n[k]; ++v) {
        int j = t->env[k][v];
        F[i][k] -= F[i][j] * F[k][j];
      }
      F[i][k] = F[i][k] / F[k][k];
    }
  }
  for (int k = 0; k < NC; ++k) {
    for (int v = 0; v < t->env_n[k]; ++v) {
      int j = t->env[k][v];
      y[k] -= F[k][j] * y[j];
    }
    y[k] /= F[k][k];
  }
  for (int k = NC - 1; k >= 0; --k) {
    for (int q = 0; q < t->col_n[k]; ++q) {
      int i = t->col[k][q];
      y[k] -= F[i][k] * s->flowv[i];
    }
    s->flowv[k] = y[k] / F[k][k];
  }
}

/* solveEquationsSor, TdsModel.cpp:2105-2180: SOR with OMEGA 1.25 from a zero start vector,
 * at most 100 sweeps while the residual norm exceeds 0.1; rows swept from the last to the
 * first, each row's off-diagonal terms from the highest column down; currents of closed
 * sections (area <= 1.01 MIN_AREA) are not computed. */
static void tds_sor(ao_synth *s, double M[NC][NC]) {
  const topo *t = &s->T;
  int active[NC];
  for (int i = 0; i < NC; ++i) active[i] = 1;
  for (int i = 0; i < NS; ++i) {
    if (s->area[i] <= 1.01 * AMIN) {
      if (t->cin[i] != -1) active[t->cin[i]] = 0;
      if (t->cout0[i] != -1) active[t->cout0[i]] = 0;
      if (t->cout1[i] != -1) active[t->cout1[i]] = 0;
    }
  }
  double *x = s->flowv;
  for (int i = 0; i < NC; ++i) x[i] = 0.0;
  int it = 0;
  double res;
  do {
    res = 0.0;
    for (int i = NC - 1; i >= 0; --i) {
      if (!active[i]) continue;
      double sum = M[i][i] * x[i];
      for (int k = t->row_n[i] - 1; k >= 0; --k) {
        int j = t->row[i][k];
        sum += x[j] * M[i][j];
      }
      double d = s->sol[i] - sum;
      res += d * d;
      x[i] += 1.25 * d / M[i][i];
    }
    it++;
  } while (it < 100 && res > 0.1 * 0.1);
  s->sor_iterations = it;
}

/* updateVariables, TdsModel.cpp:2046-2098. */
static void tds_update(ao_synth *s) {
  const double dt = s->dt;
  double c = exp(-2.0 * M_PI * NOISE_LP_HZ * dt);
  for (int i = 0; i < NC; ++i) {
    double old = s->u[i];
    s->u[i] = s->flowv[i];
    s->ur[i] = (s->u[i] - old) / (dt * TH) - (TH1 / TH) * s->ur[i];
    s->un[i] = (1.0 - c) * s->u[i] + c * s->un[i];
  }
  for (int i = 0; i < NS; ++i) {
    double net = cur_in(s, i) - cur_out(s, i);
    double old = s->p[i];
    s->p[i] = s->D[i] + s->E[i] * net;
    s->pr[i] = (s->p[i] - old) / (dt * TH) - s->pr[i] * (TH1 / TH);
    double ow = s->w[i], owr = s->wr[i];
    s->w[i] = s->pr[i] * s->alpha[i] + s->beta[i];
    s->wr[i] = (s->w[i] - ow) / (dt * TH) - owr * (TH1 / TH);
    s->wr2[i] = (s->wr[i] - owr) / (dt * TH) - s->wr2[i] * (TH1 / TH);
  }
}

/* proceedTimeStep, TdsModel.cpp:659-711. */
static double tds_step(ao_synth *s) {
  tds_prepare(s);
  memset(s->mat, 0, sizeof s->mat);
  tds_matrix(s, s->mat, s->sol);
  if (s->opt.solver == 1) tds_sor(s, s->mat);
  else tds_cholesky(s, s->mat);
  tds_update(s);
  double f = 0.0;
  int t0 = S_LAST_MOUTH, t1 = S_LAST_NOSE;
  if (s->T.cout0[t0] != -1) f += s->u[s->T.cout0[t0]];
  if (s->T.cout1[t0] != -1) f += s->u[s->T.cout1[t0]];
  if (s->T.cout0[t1] != -1) f += s->u[s->T.cout0[t1]];
  if (s->T.cout1[t1] != -1) f += s->u[s->T.cout1[t1]];
  if (s->opt.radiation_from_skin) f += iir_run(&s->tone, s->p[S_PHARYNX0]);
  s->position++;
  return f;
}

/* ---------------------------------------------------------------------------
 * Synthesizer driver, Synthesizer.cpp:515-639 (+ the state reset of :231-250).
 * ------------------------------------------------------------------------- */
ao_synth *ao_create(double fs_hz, uint32_t seed, const ao_options *opt) {
  ao_synth *s = (ao_synth *)calloc(1, sizeof(ao_synth));
  if (!s) return NULL;
  topo_build(&s->T);
  if (opt) s->opt = *opt; else ao_default_options(&s->opt);
  s->fs = fs_hz;
  s->dt = 1.0 / fs_hz;
  ao_rng_seed(&s->rng, seed);
  tube_init(s);
  for (int i = 0; i < NS; ++i) { s->dip[i].cutoff = 3000.0; }
  s->lips.cutoff = 3000.0;
  /* glottalToneFilter coefficients, TdsModel.cpp:494-510, 544 */
  static const double TA[5] = {5.027640021717718e-007, -7.995535578908732e-007, 2.967895557191014e-007, 0.0, 0.0};
  static const double TB[5] = {0.0, 3.986308869708467, -5.959669638387298, 3.960408461107104, -0.987047716233603};
  iir_clear(&s->tone);
  s->tone.order = 4;
  for (int i = 0; i <= 4; ++i) { s->tone.a[i] = TA[i]; s->tone.b[i] = TB[i]; }
  iir_reset(&s->tone);
  /* transglottalPressureFilter (TdsModel.cpp:474, 50 Hz Chebyshev at the simulation rate) and
   * the transvelar coupling filters H1, H2 (:488-533) */
  iir_clear(&s->tglot);
  chebyshev_design(50.0 / fs_hz, 0, 4, s->tglot.a, s->tglot.b, &s->tglot.order);
  iir_reset(&s->tglot);
  static const double VA2[5] = {6.589309727087047e-004, -0.001972281980771, 0.001968000742164,
                                -6.546497341015677e-004, 0.0};
  iir_clear(&s->tvel1);
  iir_clear(&s->tvel2);
  s->tvel1.order = s->tvel2.order = 4;
  for (int i = 0; i <= 4; ++i) {
    s->tvel1.a[i] = TA[i]; s->tvel1.b[i] = TB[i];
    s->tvel2.a[i] = VA2[i]; s->tvel2.b[i] = TB[i];
  }
  iir_reset(&s->tvel1);
  iir_reset(&s->tvel2);
  iir_clear(&s->outf);
  chebyshev_design(7000.0 / fs_hz, 0, 8, s->outf.a, s->outf.b, &s->outf.order);
  iir_reset(&s->outf);
  s->gp[0] = 120.0; s->gp[1] = 10000.0; s->gp[2] = 0.01; s->gp[3] = 0.01; s->gp[4] = 0.0; s->gp[5] = -40.0;
  return s;
}

void ao_destroy(ao_synth *s) { free(s); }

int ao_synthesize_call(ao_synth *s, const ao_frame *fr, int n, double *out) {
  if (!s->latched) {
    s->prev = *fr;
    s->latched = 1;
    return 0;
  }
  if (n < 1) n = 1;
  for (int i = 0; i < n; ++i) {
    double ratio = (double)i / (double)n;
    double r1 = 1.0 - ratio;
    tube_interpolate(s, &s->prev, fr, ratio);
    for (int k = 0; k < 6; ++k) s->gp[k] = r1 * s->prev.glottis[k] + ratio * fr->glottis[k];
    double gl[2], ga[2];
    if (s->opt.glottis_model == 1) tm_geometry(s, gl, ga);
    else glottis_geometry(s, gl, ga);
    for (int k = 0; k < 2; ++k) {
      int sec = S_GLOT_LO + k;
      s->len[sec] = gl[k];
      s->area[sec] = clamp_amin(ga[k]);
      s->vol[sec] = s->area[sec] * s->len[sec];
    }
    /* TriangularGlottis::getAspirationStrength_dB = control 5; the two-mass model keeps the
     * base class default (Glottis.cpp:11-16) */
    s->aspiration_db = (s->opt.glottis_model == 1) ? -40.0 : s->gp[5];
    /* setTube (TdsModel.cpp:552-584) copies the tube; our TDS arrays alias it. */
    s->teeth_tds = s->teeth;
    s->asp_tds = s->aspiration_db;
    s->p_amp = s->gp[1];
    double pg[4] = {s->p[S_LAST_TRACHEA], s->p[S_GLOT_LO], s->p[S_GLOT_UP], s->p[S_PHARYNX0]};
    if (s->opt.glottis_model == 1) tm_step(s, 1.0 / s->fs, pg);
    else glottis_step(s, 1.0 / s->fs, pg);
    double flow = tds_step(s);
    int k = s->position & 255;
    s->flow_ring[k] = flow;
    double op = (s->flow_ring[k] - s->flow_ring[(k - 1) & 255]) / s->dt;
    double y = iir_run(&s->outf, op);
    double smp = y * 0.004;
    out[i] = smp / 32767;
  }
  s->prev = *fr;
  return n;
}

int ao_position(const ao_synth *s) { return s->position; }
void ao_get_pressures(const ao_synth *s, double *p) { memcpy(p, s->p, sizeof s->p); }
void ao_get_currents(const ao_synth *s, double *u) { memcpy(u, s->u, sizeof s->u); }
long ao_rng_calls(const ao_synth *s) { return s->rng_calls; }

void ao_get_state(const ao_synth *s, double *buf, int *len) {
  int n = 0;
  for (int i = 0; i < NS; ++i) buf[n++] = s->p[i];
  for (int i = 0; i < NS; ++i) buf[n++] = s->pr[i];
  for (int i = 0; i < NS; ++i) buf[n++] = s->w[i];
  for (int i = 0; i < NS; ++i) buf[n++] = s->wr[i];
  for (int i = 0; i < NS; ++i) buf[n++] = s->wr2[i];
  for (int i = 0; i < NC; ++i) buf[n++] = s->u[i];
  for (int i = 0; i < NC; ++i) buf[n++] = s->ur[i];
  for (int i = 0; i < NC; ++i) buf[n++] = s->un[i];
  for (int i = S_PHARYNX0; i <= S_LAST_MOUTH; ++i) buf[n++] = s->dip[i].amp;
  buf[n++] = s->lips.amp;
  buf[n++] = s->gbf;
  buf[n++] = s->relx[0][s->gpos & 3];
  buf[n++] = s->relx[1][s->gpos & 3];
  *len = n;
}

long ao_synthesize_utterance(const ao_frame *frames, int F, int hop, uint32_t seed, double fs,
                             const ao_options *opt, double *out) {
  ao_synth *s = ao_create(fs, seed, opt);
  if (!s) return -1;
  long n = 0;
  ao_synthesize_call(s, &frames[0], hop, NULL);
  for (int k = 1; k < F; ++k) n += ao_synthesize_call(s, &frames[k], hop, out + n);
  ao_destroy(s);
  return n;
}

/* ---------------------------------------------------------------------------
 * OneDimAreaFunction (OneDimAreaFunction.cpp:23-58, 75-138).
 * Parameter order: Llar Alar powLar xp Ap powP xc Ac powC xa Aa powA xin Ain Lvt Alip.
 * ------------------------------------------------------------------------- */
enum { P_LLAR, P_ALAR, P_POWLAR, P_XP, P_AP, P_POWP, P_XC, P_AC, P_POWC, P_XA, P_AA, P_POWA,
       P_XIN, P_AIN, P_LVT, P_ALIP };

double ao_af_area(const double *p, double x) {
  double a;
  if (x <= p[P_LLAR]) a = p[P_ALAR];
  else if (x <= p[P_XP])
    a = (p[P_AP] + p[P_ALAR]) / 2 + (p[P_AP] - p[P_ALAR]) / 2 *
        cos(M_PI * pow((p[P_XP] - x) / (p[P_XP] - p[P_LLAR]), p[P_POWLAR]));
  else if (x <= p[P_XC])
    a = (p[P_AC] + p[P_AP]) / 2 + (p[P_AC] - p[P_AP]) / 2 *
        cos(M_PI * pow((p[P_XC] - x) / (p[P_XC] - p[P_XP]), p[P_POWP]));
  else if (x <= p[P_XA])
    a = (p[P_AA] + p[P_AC]) / 2 + (p[P_AA] - p[P_AC]) / 2 *
        cos(M_PI * pow((p[P_XA] - x) / (p[P_XA] - p[P_XC]), p[P_POWC]));
  else if (x <= p[P_XIN])
    a = (p[P_AIN] + p[P_AA]) / 2 + (p[P_AIN] - p[P_AA]) / 2 *
        cos(M_PI * pow((p[P_XIN] - x) / (p[P_XIN] - p[P_XA]), p[P_POWA]));
  else a = p[P_ALIP];
  return a < 0.0 ? 0.0 : a;
}

void ao_af_to_frame(const double *p, ao_frame *f) {
  double w = p[P_LVT] / 40;
  double step = w * 0.01;
  double x = 0.0;
  for (int i = 0; i < 40; ++i) {
    double mn = DBL_MAX;
    while (x < (i + 1) * w) {
      double a = ao_af_area(p, x);
      if (a < mn) mn = a;
      x += step;
    }
    f->length_cm[i] = w;
    f->area_cm2[i] = mn;
    f->laterality[i] = 0.0;
    if (x <= p[P_XP]) f->articulator[i] = ART_OTHER;
    else if (x <= p[P_XIN] && x + w < p[P_XIN]) f->articulator[i] = ART_TONGUE;
    else if (x <= p[P_XIN]) f->articulator[i] = ART_LOWER_INCISORS;
    else f->articulator[i] = ART_LOWER_LIP;
  }
  f->teeth_position_cm = p[P_XIN];
}

/* ---- Synthesizer::playTargetSequence (Synthesizer.cpp:1299-1422) --------------------- */

/* OneDimAreaFunction::reset, the schwa shape init() latches (OneDimAreaFunction.cpp:281-350). */
static const double AO_SCHWA[16] = {2.0, 1.0, 1.0, 3.02, 5.609, 1.0, 5.92, 2.879, 1.0, 8.48, 4.238, 1.0,
                                    15.31, 0.701, 16.44, 1.65};

void ao_target_default(ao_target_cfg *c) {
  static const double st[4] = {0.2, 0.05, 0.2, 0.1}, tr[3] = {0.05, 0.05, 0.05};
  static const double f0[4] = {100, 115, 105, 80};               /* Synthesizer.cpp:1311 */
  static const double g[6] = {120.0, 10000.0, 0.01, 0.01, 0.0, -40.0}; /* controlParam after reset() */
  memcpy(c->stationary_s, st, sizeof st);
  memcpy(c->transition_s, tr, sizeof tr);
  memcpy(c->f0_hz, f0, sizeof f0);
  c->lung_pressure_dpa = 8000.0;                                   /* sensorDataToGlottisParams :903 */
  memcpy(c->glottis, g, sizeof g);
}

/* boundary_s[0..6] of :1318-1326, summed left to right as the reference writes them. */
static void ao_target_bounds(const ao_target_cfg *c, double *b) {
  const double *s = c->stationary_s, *t = c->transition_s;
  b[0] = s[0];
  b[1] = s[0] + t[0];
  b[2] = s[0] + t[0] + s[1];
  b[3] = s[0] + t[0] + s[1] + t[1];
  b[4] = s[0] + t[0] + s[1] + t[1] + s[2];
  b[5] = s[0] + t[0] + s[1] + t[1] + s[2] + t[2];
  b[6] = s[0] + t[0] + s[1] + t[1] + s[2] + t[2] + s[3];
}

long ao_target_num_samples(const ao_target_cfg *c, double fs) {
  double b[7];
  ao_target_bounds(c, b);
  return (long)(int)(fs * b[6]);  /* int numSamples = SAMPLING_RATE * totalTime_s (:1328) */
}

/* interpolateParameters (:1286-1294) */
static void ao_interp(const double *p0, const double *p1, double *px, double t0, double t1, double tx) {
  for (int i = 0; i < 16; ++i)
    px[i] = (p1[i] - p0[i]) / 2 * cos((t1 - tx) / (t1 - t0) * M_PI) + (p1[i] + p0[i]) / 2;
}

/* The lung-pressure statements of :1333-1346 and :1399-1403 for sample i (before the
 * fade-out check). */
static double ao_fade_in(double P, double fs, long i) {
  if (i < (double)0.05 * (double)fs) return 0.0;
  return P / 2 * cos((0.1 * fs - i) / (0.05 * fs) * M_PI) + P / 2;
}

static double ao_pressure(const ao_target_cfg *c, double fs, double total, long i) {
  const double P = c->lung_pressure_dpa;
  double v;
  if (i < (double)0.1 * (double)fs) {
    v = ao_fade_in(P, fs, i);
  } else {
    /* held: the value the last sample below 0.1 fs set, or P if none did */
    long j = (long)ceil((double)0.1 * (double)fs);  /* the largest j with j < 0.1 fs */
    while (j >= 0 && !(j < (double)0.1 * (double)fs)) --j;
    while ((double)(j + 1) < (double)0.1 * (double)fs) ++j;
    v = (j >= 0) ? ao_fade_in(P, fs, j) : P;
  }
  if (i > (double)(total - 0.1) * (double)fs)  /* the reference's fade-out, denominator as written */
    v = -P / 2 * cos((total * fs - i) / (total - 0.1 * fs) * M_PI) + P / 2;
  return v;
}

static double ao_f0(const ao_target_cfg *c, const double *b, double fs, long i) {
  const double *f = c->f0_hz;
  if (i < (double)b[1] * fs)
    return (f[0] + f[1]) / 2 + (f[1] - f[0]) / 2 * cos((b[1] * fs - i) / (b[1] * fs) * M_PI);
  if (i < (double)b[3] * fs)
    return (f[2] + f[1]) / 2 + (f[2] - f[1]) / 2 * cos((b[3] * fs - i) / ((b[3] - b[1]) * fs) * M_PI);
  return (f[3] + f[2]) / 2 + (f[3] - f[2]) / 2 * cos((b[6] * fs - i) / ((b[6] - b[3]) * fs) * M_PI);
}

/* currentParams of sample i (:1364-1397); shapes = 4 x 16 targets. */
static void ao_target_params(const double *shapes, const double *b, double fs, long i, double *p) {
  const double *s0 = shapes, *s1 = shapes + 16, *s2 = shapes + 32, *s3 = shapes + 48;
  if (i <= b[0] * fs) memcpy(p, s0, 16 * sizeof(double));
  else if (i <= b[1] * fs) ao_interp(s0, s1, p, b[0] * fs, b[1] * fs, i);
  else if (i <= b[2] * fs) memcpy(p, s1, 16 * sizeof(double));
  else if (i <= b[3] * fs) ao_interp(s1, s2, p, b[2] * fs, b[3] * fs, i);
  else if (i <= b[4] * fs) memcpy(p, s2, 16 * sizeof(double));
  else if (i <= b[5] * fs) ao_interp(s2, s3, p, b[4] * fs, b[5] * fs, i);
  else memcpy(p, s3, 16 * sizeof(double));  /* i <= b[6] fs for every i < numSamples */
}

void ao_target_frames(const double *shapes, const ao_target_cfg *c, double fs, long k0, long n, ao_frame *out) {
  double b[7];
  ao_target_bounds(c, b);
  for (long k = 0; k < n; ++k) {
    const long g = k0 + k;
    ao_frame *f = out + k;
    memset(f, 0, sizeof *f);
    if (g == 0) {  /* init(): the schwa tube and the glottis parameters of reset() */
      ao_af_to_frame(AO_SCHWA, f);
      for (int q = 0; q < 6; ++q) f->glottis[q] = c->glottis[q];
    } else {       /* sample i = g - 1: synthesizeSignalTds(tube_i, glottis_i, 1) */
      const long i = g - 1;
      double p[16];
      ao_target_params(shapes, b, fs, i, p);
      ao_af_to_frame(p, f);
      f->glottis[0] = ao_f0(c, b, fs, i);
      f->glottis[1] = ao_pressure(c, fs, b[6], i);
      for (int q = 2; q < 6; ++q) f->glottis[q] = c->glottis[q];
    }
    f->velum_opening_cm2 = 0.0;  /* the Synthesizer's tube keeps Tube()'s closed velum */
  }
}

/* Synthesizer.cpp:955-973: audioBuffer->setValue(pos, newSignal[i] * SHRT_MAX) stores into
 * a Signal16 (signed short), then the two clipping branches overwrite out-of-range values. */
void ao_to_int16(const double *x, long n, int16_t *out) {
  for (long i = 0; i < n; ++i) {
    const double v = x[i];
    int16_t s;
    if (v != v) s = 0;
    else if (v > 1.0) s = 32767;
    else if (v < -1.0) s = -32768;
    else s = (int16_t)(int)(v * 32767.0);
    out[i] = s;
  }
}
