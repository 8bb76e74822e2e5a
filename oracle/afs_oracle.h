/*
 * afs_oracle.h -- CPU restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (areafunctionsynthesis_amd/,
 * include/) links, loads or calls this code.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may use it, and only as the checker.
 *
 * What it restates (reference = /root/reference, file:line):
 *   Synthesizer::synthesizeSignalTds          src/Backend/Synthesizer.cpp:515-639
 *   Tube (static geometry, interpolate, ...)  src/Backend/Tube.cpp:46-654
 *   TriangularGlottis (calcGeometry/incTime)  src/Backend/TriangularGlottis.cpp:154-576
 *   TdsModel (proceedTimeStep and stages)     src/Backend/TdsModel.cpp:67-2385
 *   IirFilter (run, one-pole, Chebyshev)      src/Backend/IirFilter.cpp:47-432
 *   glibc random_r TYPE_3 (rand()/srand())    glibc 2.35 stdlib/random_r.c (the
 *                                             reference calls rand() at
 *                                             src/Backend/TdsModel.cpp:1690-1692)
 *   TwoMassModel (alternative glottis)        src/Backend/TwoMassModel.cpp:1-497
 *   OneDimAreaFunction (area fn -> tube)      src/Backend/OneDimAreaFunction.cpp:23-138
 *   Synthesizer::playTargetSequence           src/Backend/Synthesizer.cpp:1286-1422
 *   int16 output ring                         src/Backend/Synthesizer.cpp:955-973
 *
 * Parity pin: the restatement is checked bit-for-bit against oracle/_ref, a build of
 * the reference's own TdsModel/Tube/TriangularGlottis/IirFilter sources driven by
 * oracle/ref_harness.cpp (tests/test_oracle_vs_ref.py), and against the committed
 * golden vectors in tests/golden/ that the same reference build produced.
 * OneDimAreaFunction and Synthesizer.cpp are not buildable from the reference (wxWidgets /
 * portaudio); the area-function and target-sequence rows are pinned by the restatement
 * and its tests only.
 */
#ifndef AFS_ORACLE_H
#define AFS_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AO_NUM_PM 40          /* Tube::NUM_PHARYNX_MOUTH_SECTIONS, Tube.h:56 */
#define AO_NUM_GLOTTIS_PARAMS 6 /* TriangularGlottis::NUM_CONTROL_PARAMS */

/* One synthesis frame = the arguments of one synthesizeSignalTds() call:
 * the dynamic part of the Tube plus the six glottis control parameters.
 * Byte layout is identical to afs_frame in include/afs.h (1072 bytes). */
typedef struct ao_frame {
  double area_cm2[AO_NUM_PM];
  double length_cm[AO_NUM_PM];
  double laterality[AO_NUM_PM];
  double teeth_position_cm;
  double velum_opening_cm2;
  double glottis[AO_NUM_GLOTTIS_PARAMS];
  uint8_t articulator[AO_NUM_PM];
  uint8_t pad_[8];
} ao_frame;

/* TdsModel::Options (TdsModel.h:83-95); defaults of TdsModel.cpp:35-44. */
typedef struct ao_options {
  int turbulence_losses;        /* 1 */
  int soft_walls;               /* 1 */
  int generate_noise_sources;   /* 1 */
  int radiation_from_skin;      /* 1 */
  int piriform_fossa;           /* 0 */
  int inner_length_corrections; /* 1 */
  int transvelar_coupling;      /* 0 */
  int glottis_loss;             /* 0 STANDARD, 1 VAN_DEN_BERG, 2 VARIABLE (Fulcher 2011) */
  int solver;                   /* 0 CHOLESKY_FACTORIZATION, 1 SOR_GAUSS_SEIDEL */
  int glottis_model;            /* 0 TriangularGlottis (the Synthesizer's), 1 TwoMassModel */
  double flow_separation_area_ratio; /* 1.0 */
} ao_options;

/* getGlottalEntranceLossCoeffFlucher2011(pressure_dPa, d_cm) (TdsModel.cpp:1048-1092). */
double ao_fulcher_kent(double pressure_dPa, double d_cm);

void ao_default_options(ao_options *o);

/* Opaque single-utterance synthesizer (one Synthesizer + TdsModel + glottis). */
typedef struct ao_synth ao_synth;

ao_synth *ao_create(double fs_hz, uint32_t seed, const ao_options *opt);
void ao_destroy(ao_synth *s);
/* synthesizeSignalTds(newTube, glottis, n, out): the first call only latches the
 * frame (Synthesizer.cpp:522-532) and returns 0; later calls produce max(n,1)
 * samples into out and return that count. */
int ao_synthesize_call(ao_synth *s, const ao_frame *frame, int n, double *out);

/* Introspection after the latest sample (for per-step fixtures). */
int ao_position(const ao_synth *s);
void ao_get_pressures(const ao_synth *s, double *p93);
void ao_get_currents(const ao_synth *s, double *u97);
void ao_get_state(const ao_synth *s, double *buf, int *len); /* flat dump */
long ao_rng_calls(const ao_synth *s);

/* Whole utterance: latch frames[0], then (F-1) calls of hop samples.
 * out must hold (F-1)*hop doubles.  Returns the number of samples. */
long ao_synthesize_utterance(const ao_frame *frames, int num_frames, int hop,
                             uint32_t seed, double fs_hz, const ao_options *opt,
                             double *out);

/* glibc TYPE_3 generator restatement (srand/rand semantics). */
typedef struct ao_rng { int32_t r[31]; int f; } ao_rng;
void ao_rng_seed(ao_rng *g, uint32_t seed);
int32_t ao_rng_next(ao_rng *g);

/* OneDimAreaFunction: 16 parameters (OneDimAreaFunction.h:34-43) -> the pharynx/
 * mouth part of a frame (area, length, articulator, laterality, teeth).
 * Velum and glottis fields are left untouched. */
void ao_af_to_frame(const double params16[16], ao_frame *f);
double ao_af_area(const double params16[16], double x_cm);

/* Synthesizer::playTargetSequence (Synthesizer.cpp:1299-1422) as a hop-1 frame trajectory:
 * frame 0 is init()'s latch (the schwa of OneDimAreaFunction::reset and reset()'s glottis
 * parameters), frame k >= 1 holds sample k-1's tube (interpolateParameters, cosine) and
 * glottis controls (F0 contour, lung-pressure fade-in/hold/fade-out as written).  Sample i
 * of the utterance is synthesizeSignalTds(frame i+1, ..., 1), i.e. it plays frame i. */
typedef struct ao_target_cfg {
  double stationary_s[4];
  double transition_s[3];
  double f0_hz[4];
  double lung_pressure_dpa;
  double glottis[6];
} ao_target_cfg;
void ao_target_default(ao_target_cfg *c);
long ao_target_num_samples(const ao_target_cfg *c, double fs);
void ao_target_frames(const double *shapes4x16, const ao_target_cfg *c, double fs, long k0, long n, ao_frame *out);

/* IirFilter::createChebyshev (IirFilter.cpp:286-432): a[0..order], b[0..order]. */
int ao_chebyshev(double cutoff_ratio, int highpass, int poles, double *a, double *b);

/* Synthesizer::synthesizeSegment's int16 ring (Synthesizer.cpp:955-973): short(x*SHRT_MAX)
 * (truncation), x > 1 -> SHRT_MAX, x < -1 -> SHRT_MIN; NaN -> 0 (the x86 conversion). */
void ao_to_int16(const double *x, long n, int16_t *out);

#ifdef __cplusplus
}
#endif
#endif
