// ref_harness.cpp -- drives the REFERENCE's own hot-path classes.
//
// TEST INFRASTRUCTURE ONLY.  Built by oracle/Makefile together with the reference's
// unmodified sources TdsModel.cpp, Tube.cpp, TriangularGlottis.cpp, Glottis.cpp,
// IirFilter.cpp, XmlNode.cpp, Dsp.cpp and Signal.cpp, compiled where they lie under
// /root/reference/src/Backend, into oracle/_ref/libafsref.so.  No reference source
// is copied; nothing is stubbed.  Only tests/ (golden-vector generation, restatement
// pinning) and bench.py's cpu_baseline leg load the result.
//
// The Synthesizer class itself (Synthesizer.cpp) needs wxWidgets and portaudio and is
// not buildable here, so the per-sample driver below restates
// Synthesizer::synthesizeSignalTds (Synthesizer.cpp:515-639) on top of the
// reference's public TdsModel / TriangularGlottis / Tube / IirFilter API.  The
// sampling rate is a run-time argument: TdsModel::timeStep is a public member
// (TdsModel.h:228) that the harness sets after construction, so 44.1 kHz runs use the
// unmodified reference code as well.
#include <climits>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>

#include <unistd.h>

#include "IirFilter.h"
#include "TdsModel.h"
#include "TriangularGlottis.h"
#include "Tube.h"
#include "TwoMassModel.h"

extern "C" {
#include "afs_oracle.h"  // only for the ao_frame record layout
}

static long g_rand_calls = 0;
extern "C" int __real_rand(void);
extern "C" int __wrap_rand(void) {
  ++g_rand_calls;
  return __real_rand();
}

namespace {

struct RefVoice {
  TdsModel tds;
  TriangularGlottis triangular;
  TwoMassModel twoMass;  // TwoMassModel.cpp: in the reference's sources, not in its executable
  Glottis *glottis = &triangular;
  Tube tube;       // Synthesizer::tube
  Tube prevTube;   // Synthesizer::prevTube
  Tube newTube;    // the caller-owned frame tube
  double prevGlottis[8] = {0};
  bool latched = false;
  IirFilter outputPressureFilter;
  double outputFlow[256] = {0};  // zero-initialised (Synthesizer.cpp:617 reads [0] first)
  double fs = 22050.0;

  RefVoice(double fs_hz, unsigned seed, int glottis_model = 0) : fs(fs_hz) {
    if (glottis_model == 1) glottis = &twoMass;
    tds.timeStep = 1.0 / fs_hz;
    outputPressureFilter.createChebyshev(7000.0 / fs_hz, false, 8);
    tds.resetMotion();        // Synthesizer::reset, Synthesizer.cpp:231-250
    // resetMotion designs the transglottal-pressure low-pass at 50 Hz / TDS_SAMPLING_RATE
    // (TdsModel.cpp:474); at a run-time rate it is redesigned for that rate, as the
    // reference compiled with SAMPLING_RATE = fs would (identical at 22050 Hz).
    tds.transglottalPressureFilter.createChebyshev(50.0 / fs_hz, false, 4);
    tds.transglottalPressureFilter.resetBuffers();
    glottis->resetMotion();
    outputPressureFilter.resetBuffers();
    srand(seed);
  }

  void loadFrame(const ao_frame *f) {
    double len[40], area[40], lat[40];
    Tube::Articulator art[40];
    for (int i = 0; i < 40; ++i) {
      len[i] = f->length_cm[i];
      area[i] = f->area_cm2[i];
      lat[i] = f->laterality[i];
      art[i] = static_cast<Tube::Articulator>(f->articulator[i]);
    }
    newTube.setPharynxMouthGeometry(len, area, art, lat, f->teeth_position_cm);
    newTube.teethPosition_cm = f->teeth_position_cm;
    newTube.setVelumOpening(f->velum_opening_cm2);
  }

  // Synthesizer::synthesizeSignalTds, Synthesizer.cpp:515-639.
  int call(const ao_frame *f, int n, double *out) {
    loadFrame(f);
    const double *g = f->glottis;
    const int ng = (int)glottis->controlParam.size();
    if (!latched) {
      prevTube = newTube;
      for (int i = 0; i < ng; ++i) prevGlottis[i] = g[i];
      latched = true;
      return 0;
    }
    if (n < 1) n = 1;
    for (int i = 0; i < n; ++i) {
      double ratio = (double)i / (double)n;
      double ratio1 = 1.0 - ratio;
      tube.interpolate(&prevTube, &newTube, ratio);
      for (int k = 0; k < ng; ++k) glottis->controlParam[k].x = ratio1 * prevGlottis[k] + ratio * g[k];
      glottis->calcGeometry();
      double l[2], a[2];
      glottis->getTubeData(l, a);
      tube.setGlottisGeometry(l, a);
      tube.setAspirationStrength(glottis->getAspirationStrength_dB());
      tds.setTube(&tube, tds.getSampleIndex() != 0);
      tds.setFlowSource(0.0, -1);
      tds.setPressureSource(glottis->controlParam[Glottis::PRESSURE].x, Tube::FIRST_TRACHEA_SECTION);
      double p[4] = {tds.getSectionPressure(Tube::LAST_TRACHEA_SECTION),
                     tds.getSectionPressure(Tube::LOWER_GLOTTIS_SECTION),
                     tds.getSectionPressure(Tube::UPPER_GLOTTIS_SECTION),
                     tds.getSectionPressure(Tube::FIRST_PHARYNX_SECTION)};
      glottis->incTime(1.0 / fs, p);
      double flow = tds.proceedTimeStep();
      int pos = tds.getSampleIndex();
      int k = pos & 255;
      outputFlow[k] = flow;
      double op = (outputFlow[k] - outputFlow[(k - 1) & 255]) / tds.timeStep;
      double y = outputPressureFilter.getOutputSample(op);
      double s = y * 0.004;
      out[i] = s / SHRT_MAX;
    }
    prevTube = newTube;
    for (int i = 0; i < ng; ++i) prevGlottis[i] = g[i];
    return n;
  }
};

}  // namespace

extern "C" {

void *afsref_create(double fs_hz, unsigned seed) { return new RefVoice(fs_hz, seed); }
void afsref_destroy(void *v) { delete static_cast<RefVoice *>(v); }
int afsref_call(void *v, const ao_frame *f, int n, double *out) {
  return static_cast<RefVoice *>(v)->call(f, n, out);
}
int afsref_position(void *v) { return static_cast<RefVoice *>(v)->tds.getSampleIndex(); }
void afsref_pressures(void *v, double *p) {
  RefVoice *r = static_cast<RefVoice *>(v);
  for (int i = 0; i < Tube::NUM_SECTIONS; ++i) p[i] = r->tds.tubeSection[i].pressure;
}
void afsref_currents(void *v, double *u) {
  RefVoice *r = static_cast<RefVoice *>(v);
  for (int i = 0; i < TdsModel::NUM_BRANCH_CURRENTS; ++i) u[i] = r->tds.branchCurrent[i].magnitude;
}
long afsref_rand_calls(void) { return g_rand_calls; }

// One utterance end to end: latch frames[0], then (F-1) calls of hop samples.
// opt (optional): every field of TdsModel::Options (TdsModel.h:83-95), in ao_options layout.
long afsref_utterance_opt(const ao_frame *frames, int F, int hop, unsigned seed, double fs, double *out,
                          const ao_options *opt) {
  RefVoice *v = new RefVoice(fs, seed, opt ? opt->glottis_model : 0);
  if (opt) {
    TdsModel::Options &o = v->tds.options;
    o.turbulenceLosses = opt->turbulence_losses != 0;
    o.softWalls = opt->soft_walls != 0;
    o.generateNoiseSources = opt->generate_noise_sources != 0;
    o.radiationFromSkin = opt->radiation_from_skin != 0;
    o.piriformFossa = opt->piriform_fossa != 0;
    o.innerLengthCorrections = opt->inner_length_corrections != 0;
    o.transvelarCoupling = opt->transvelar_coupling != 0;
    o.glottisLossOption = opt->glottis_loss == 1   ? TdsModel::ENTRANCE_LOSS_VAN_DEN_BERG
                          : opt->glottis_loss == 2 ? TdsModel::VARIABLE_ENTRANCE_LOSS
                                                   : TdsModel::STANDARD_ENTRANCE_LOSS;
    o.flowSeparationAreaRatio = opt->flow_separation_area_ratio;
    o.solverType = opt->solver == 1 ? TdsModel::SOR_GAUSS_SEIDEL : TdsModel::CHOLESKY_FACTORIZATION;
  }
  long n = 0;
  v->call(&frames[0], hop, nullptr);
  for (int k = 1; k < F; ++k) n += v->call(&frames[k], hop, out + n);
  delete v;
  return n;
}

long afsref_utterance(const ao_frame *frames, int F, int hop, unsigned seed, double fs, double *out) {
  RefVoice *v = new RefVoice(fs, seed);
  long n = 0;
  v->call(&frames[0], hop, nullptr);
  for (int k = 1; k < F; ++k) n += v->call(&frames[k], hop, out + n);
  delete v;
  return n;
}

// The reference's own Fulcher et al. (2011) Table I printout
// (TdsModel::checkGlottalEntranceLossCoeffFlucher2011, TdsModel.cpp:1100-1181), captured from
// stdout into buf.  Returns the number of bytes.
int afsref_fulcher_table(char *buf, int cap) {
  TdsModel tds;
  fflush(stdout);
  int fds[2];
  if (pipe(fds) != 0) return -1;
  int saved = dup(1);
  dup2(fds[1], 1);
  tds.checkGlottalEntranceLossCoeffFlucher2011();
  fflush(stdout);
  dup2(saved, 1);
  close(saved);
  close(fds[1]);
  int n = 0, r;
  while (n < cap - 1 && (r = (int)read(fds[0], buf + n, (size_t)(cap - 1 - n))) > 0) n += r;
  close(fds[0]);
  buf[n] = 0;
  return n;
}

int afsref_chebyshev(double ratio, int highpass, int poles, double *a, double *b) {
  IirFilter f;
  f.createChebyshev(ratio, highpass != 0, poles);
  for (int i = 0; i <= f.order; ++i) { a[i] = f.a[i]; b[i] = f.b[i]; }
  return f.order;
}

// Synthesizer::synthesizeSegment's output stage (Synthesizer.cpp:955-973) on the reference's
// own Signal16 ring: the same three statements per sample.
void afsref_to_int16(const double *x, int n, short *out) {
  Signal16 buf(n);
  for (int i = 0; i < n; ++i) {
    buf.setValue(i, (double)x[i] * SHRT_MAX);
    if (x[i] > 1.0) buf.setValue(i, SHRT_MAX);
    if (x[i] < -1.0) buf.setValue(i, SHRT_MIN);
    out[i] = buf.getValue(i);
  }
}

void afsref_glibc_rand(unsigned seed, int n, int *out) {
  srand(seed);
  for (int i = 0; i < n; ++i) out[i] = rand();
}

}  // extern "C"
