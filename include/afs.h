/*
 * afs.h -- C ABI of the MI355X batched area-function synthesizer (libafs.so).
 *
 * This is the drop-in boundary for the reference's synthesis hot path.  The reference
 * has no FFI layer; its callers use the C++ class API, and every entry point below
 * names the reference interface it replaces:
 *
 *   afs_session_synthesize  <- Synthesizer::synthesizeSignalTds(Tube*, double*, int, double*)
 *                              src/Backend/Synthesizer.h:161-162, Synthesizer.cpp:515-639
 *                              (together with TdsModel::setTube / setFlowSource /
 *                              setPressureSource / proceedTimeStep, TdsModel.h:267-271, and
 *                              Glottis::calcGeometry / getTubeData / incTime, Glottis.h:77-82)
 *   afs_session_reset       <- Synthesizer::reset (Synthesizer.cpp:231-250: TdsModel::resetMotion,
 *                              TriangularGlottis::resetMotion, output filter reset) + srand(seed)
 *   afs_synthesize          <- the same driver run over whole trajectories: one latch call on
 *                              frame 0 then F-1 calls of `hop` samples each, as
 *                              Synthesizer::synthesizeSegment (Synthesizer.cpp:928-986) and
 *                              playTargetSequence (:1299-1422) drive it, for B utterances at once
 *   afs_af_to_frames        <- OneDimAreaFunction::calculateOneDimTubeFunction
 *                              (src/Backend/OneDimAreaFunction.cpp:75-138)
 *   afs_options             <- TdsModel::Options (src/Backend/TdsModel.h:83-95)
 *   afs_to_int16            <- the int16 audio ring of Synthesizer::synthesizeSegment
 *                              (Synthesizer.cpp:955-973, Signal16 = short, Signal.h:19)
 *   afs_play_target_sequences <- Synthesizer::playTargetSequence (Synthesizer.cpp:1299-1422)
 *                              with interpolateParameters (:1286-1294), for B utterances
 *   afs_multi_synthesize    <- the same whole-trajectory driver over several GPUs of one node,
 *   afs_comm_*, afs_gather_pcm  the int16 audio (Synthesizer.cpp:955-973) gathered to the first
 *                              GPU over RCCL (the reference has one Synthesizer per process and
 *                              no collectives; this is the only exchange the batch needs)
 *
 * Errors: the reference prints and continues (TdsModel.cpp:1832,1849,1898,2267); here every
 * call returns an afs_status and afs_last_error() holds a message.  Inputs are clamped exactly
 * as the reference clamps them (areas >= 0.001 cm^2, Tube.cpp:337/371/413).  Non-finite audio
 * (the reference's "matrix is not positive definite" path, TdsModel.cpp:2267) is reported per
 * utterance in the optional `nonfinite` flag array of the synthesis calls and counted in
 * afs_report.nonfinite_utterances.
 *
 * Seeds: srand() seed per utterance / voice; a NULL seed array seeds utterance u with u + 1.
 *
 * Memory: frames / seeds / out may be host or device (hipMalloc) pointers; the library
 * detects which.  Device state lives in the session.  One context per host thread.
 * All work is issued on the context's HIP stream (afs_set_stream) and the calls are
 * synchronous unless AFS_ASYNC is set in afs_config.flags.
 */
#ifndef AFS_H
#define AFS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AFS_ABI_VERSION 5
#define AFS_NUM_TUBE_SECTIONS 40   /* Tube::NUM_PHARYNX_MOUTH_SECTIONS (Tube.h:56-58) */
#define AFS_NUM_GLOTTIS_PARAMS 6   /* TriangularGlottis::NUM_CONTROL_PARAMS (TriangularGlottis.h:26-35) */
#define AFS_NUM_AF_PARAMS 16       /* OneDimAreaFunction::NUM_AF_PARAMS (OneDimAreaFunction.h:34-43) */

typedef enum afs_status {
  AFS_OK = 0,
  AFS_ERR_INVALID_ARGUMENT = 1,
  AFS_ERR_NO_DEVICE = 2,
  AFS_ERR_HIP = 3,
  AFS_ERR_OUT_OF_MEMORY = 4,
  AFS_ERR_UNSUPPORTED = 5
} afs_status;

/* Linear solver for the per-sample 97x97 SPD system. */
typedef enum afs_solver {
  AFS_SOLVER_CHOLESKY = 0, /* TdsModel::CHOLESKY_FACTORIZATION, same operation order (TdsModel.cpp:2231-2314):
                              one lane per utterance, the reference-order kernel (slow; for checks) */
  AFS_SOLVER_TREE = 1,     /* the default and the fastest: 16 lanes per utterance, the same system solved by an
                              LDL^T in arm order (tube tree, fewer flops), noise-source plans computed ahead */
  AFS_SOLVER_SOR = 2       /* TdsModel::SOR_GAUSS_SEIDEL, same sweep order (TdsModel.cpp:2105-2180), one lane
                              per utterance */
  /* 3 was AFS_SOLVER_SEG (a segment-aligned cooperative kernel, measured 42 % slower than TREE and
     withdrawn in ABI 5): afs_create rejects it with AFS_ERR_INVALID_ARGUMENT */
} afs_solver;

/* Glottis model driven by the synthesizer: the reference's Synthesizer uses TriangularGlottis
 * (Synthesizer.h:212-213); TwoMassModel (TwoMassModel.cpp) is the other Glottis subclass in its
 * sources.  Its six controls are f0, lung pressure, rest displacements 1/2, extra arytenoid
 * area and damping factor (afs_frame.glottis[5] is the damping factor; aspiration stays at
 * Glottis::DEFAULT_ASPIRATION_STRENGTH_DB = -40 dB). */
typedef enum afs_glottis_model {
  AFS_GLOTTIS_TRIANGULAR = 0,
  AFS_GLOTTIS_TWO_MASS = 1
} afs_glottis_model;

/* TdsModel::GlottisLossOptions (TdsModel.h:75-81). */
typedef enum afs_glottis_loss {
  AFS_ENTRANCE_LOSS_STANDARD = 0,     /* k_ent = 1 */
  AFS_ENTRANCE_LOSS_VAN_DEN_BERG = 1, /* k_ent = 1.375 */
  AFS_ENTRANCE_LOSS_VARIABLE = 2      /* Fulcher et al. 2011 (TdsModel.cpp:1019-1092) */
} afs_glottis_loss;

typedef enum afs_precision { AFS_FP64 = 0 } afs_precision;

/* Options of TdsModel (TdsModel.h:83-95), defaults of TdsModel.cpp:35-44. */
typedef struct afs_options {
  int32_t turbulence_losses;        /* 1 */
  int32_t soft_walls;               /* 1 */
  int32_t generate_noise_sources;   /* 1 */
  int32_t radiation_from_skin;      /* 1 */
  int32_t piriform_fossa;           /* 0 */
  int32_t inner_length_corrections; /* 1 */
  int32_t transvelar_coupling;      /* 0 */
  int32_t glottis_loss;             /* afs_glottis_loss, 0 */
  int32_t glottis_model;            /* afs_glottis_model, 0 (not a TdsModel option: the synthesizer's glottis) */
  double flow_separation_area_ratio; /* 1.0 */
} afs_options;

/* Calls return once their work is queued on the context's stream.  One exception: a large tree call
 * (its mixed hops' noise plans may overflow the plan budget) reads back how many plan slots K5
 * claimed, after its synthesis launches are queued (guarded on the device: they do nothing on an
 * overflow, and the call then queues its chunked path).  That wait covers the work queued before K5,
 * the previous call's synthesis included, but the device does not idle: this call's synthesis is
 * queued behind K5.  The slot order is sorted on the device, with no read-back. */
#define AFS_ASYNC 0x1u
/* Record an event pair around every kernel launch of the synthesis calls; afs_kernel_times
 * returns their summed durations (measurement only: a few microseconds per launch). */
#define AFS_PROFILE 0x2u
/* Tree solver, lanes per utterance.  By default the library picks per call (per session: at its
 * creation) from the batch: the voice kernel (64 lanes, two tube sections per lane, each utterance's
 * phases split over a pair of waves on two SIMDs: the shortest time per sample) while the batch is no
 * larger than the GPU's SIMD count, the throughput kernel (16 lanes, six sections per lane, four
 * utterances per pair of waves, two waves per SIMD) above.  These
 * flags force one of them (not both).  The two kernels evaluate the same operations per section but
 * are separate compilations: their audio agrees within the parity tolerances, not bit for bit. */
#define AFS_LANES_16 0x4u
#define AFS_LANES_64 0x8u

typedef struct afs_config {
  double sampling_rate_hz; /* reference: 22050 (Constants.h:22-26); any rate is accepted */
  int32_t precision;       /* afs_precision */
  int32_t solver;          /* afs_solver */
  int32_t device;          /* HIP device ordinal */
  uint32_t flags;          /* AFS_ASYNC | AFS_PROFILE | AFS_LANES_16 or AFS_LANES_64 */
  afs_options options;
} afs_config;

/* One frame = the arguments of one synthesizeSignalTds() call: the dynamic part of the
 * caller's Tube and the six glottis control parameters.  1072 bytes. */
typedef struct afs_frame {
  double area_cm2[AFS_NUM_TUBE_SECTIONS];   /* Tube::pharynxMouthSection[i].area_cm2 */
  double length_cm[AFS_NUM_TUBE_SECTIONS];  /* .length_cm */
  double laterality[AFS_NUM_TUBE_SECTIONS]; /* .laterality */
  double teeth_position_cm;                 /* Tube::teethPosition_cm */
  double velum_opening_cm2;                 /* argument of Tube::setVelumOpening */
  double glottis[AFS_NUM_GLOTTIS_PARAMS];   /* f0 Hz, lung pressure dPa, rest disp 1/2 cm, ary area cm^2, aspiration dB */
  uint8_t articulator[AFS_NUM_TUBE_SECTIONS]; /* Tube::Articulator (Tube.h:24-32) */
  uint8_t reserved[8];
} afs_frame;

typedef struct afs_report {
  double device_ms;              /* time of the synthesis kernels (HIP events) */
  int64_t samples;               /* audio samples produced (all utterances) */
  int32_t nonfinite_utterances;  /* utterances whose output contains NaN/Inf */
  int32_t kernel;                /* which kernel ran (implementation detail, for profiles) */
} afs_report;

typedef struct afs_ctx afs_ctx;
typedef struct afs_session afs_session;

void afs_config_default(afs_config *cfg);
const char *afs_status_string(afs_status s);
int32_t afs_abi_version(void);

/* Environment read by afs_create (studies and A/B runs; the defaults are the measured best):
 *   AFS_PLAN_DENSE=1        every hop reads K5's dense per-sample records (bit-exact plan, below)
 *   AFS_PLAN_BUDGET_MB=N    noise-plan memory per call (default 4096); past it the call runs in
 *                           launches of at most N MB of plans -- with one floor: a launch spans at
 *                           least one hop, so a hop-mode launch holds at least two hops of dense
 *                           records per row (2 x hop x 128 B x rows) even when that exceeds N MB
 *   AFS_LAUNCH_SAMPLES=N    samples per synthesis-kernel launch at most (default 65536; the state
 *                           crosses launches, the audio is the same bit for bit)
 *   AFS_XCD_ORDER=0         shared trajectories (target sequences) in utterance order instead of
 *                           the XCD-aware order
 *   AFS_SHAPE_ORDER=0       afs_synthesize's utterances in call order in the 16-lane kernel's
 *                           slots instead of sorted by the shape of their first frame (the audio
 *                           of each utterance is the same either way)
 *   AFS_NOISE_VARIANTS=0    the synthesis kernel always runs its full noise phases instead of the
 *                           lightest variant each launch's noise-source plans allow (same audio);
 *                           =2 the variants for every call (default: for calls whose batch is mostly
 *                           light or holds >= 16 waves per SIMD: DESIGN.md 2.5)
 *   AFS_PLAN_OVERLAP=1      chunked path: K5 of the next launch beside K1 of this one
 *   AFS_STAT_PRIO=0..3      when the throughput kernel's STAT waves run at the higher issue priority:
 *                           never / the solver / the first phase group and the solver / always
 *                           (default: 2 for launches of two or more rounds of workgroups per CU) */
afs_status afs_create(afs_ctx **ctx, const afs_config *cfg);
void afs_destroy(afs_ctx *ctx);
const char *afs_last_error(const afs_ctx *ctx);
/* Use this hipStream_t (passed as void*) for all work of the context; NULL = default stream. */
afs_status afs_set_stream(afs_ctx *ctx, void *hip_stream);
/* Lanes per utterance the tree solver uses for a batch of this size (AFS_LANES_*; 1 for the
 * one-lane solvers). */
int32_t afs_lanes_per_utterance(const afs_ctx *ctx, int32_t batch);
/* Name of the synthesis kernel a batch of this size runs ("tree_pair_kernel": 16 lanes per
 * utterance, two waves per SIMD; "tree_pair64_kernel": the 64-lane voice kernel as wave pairs, small
 * batches; "tree_synth_kernel": the 64-lane voice kernel one wave per utterance, or any batch of a
 * one-wave build; "lane_synth_kernel": the one-lane solvers) -- for matching profiler output.
 * Diagnostics; no reference counterpart. */
const char *afs_synthesis_kernel(const afs_ctx *ctx, int32_t batch);
afs_status afs_synchronize(afs_ctx *ctx);

/* Whole trajectories.  frames[batch][num_frames], seeds[batch] (srand() seed per utterance,
 * 0 behaves as 1 like glibc; NULL: u + 1), out[batch][(num_frames-1)*hop] doubles in [-1,1].
 * nonfinite: NULL or batch bytes (host or device), set to 1 for the utterances whose audio
 * holds a NaN or an infinity, else 0. */
afs_status afs_synthesize(afs_ctx *ctx, const afs_frame *frames, const uint32_t *seeds,
                          int32_t batch, int32_t num_frames, int32_t hop, double *out,
                          uint8_t *nonfinite, afs_report *report);
/* Diagnostics: the number of rand() calls (TdsModel.cpp:1690-1692) each utterance of the last
 * afs_synthesize / afs_play_target_sequences call made, draws[batch] (host or device).  A
 * count that differs from the reference's means a noise source switched on or off at a
 * different sample (TdsModel.cpp:1647-1666).  Tree solver only (else AFS_ERR_UNSUPPORTED). */
afs_status afs_rng_draws(afs_ctx *ctx, int32_t batch, int64_t *draws);
/* Diagnostics: the noise-source plan records the tree solver computes ahead of the time
 * loop (kernel K5; AFS_PLAN_WORDS u64 words per sample, layout in csrc/tree_plan.h) for samples
 * [s_begin, s_end) of frames[rows][num_frames] at this hop: plans[rows][s_end - s_begin]
 * [AFS_PLAN_WORDS] (host or device).  Everything calcNoiseSources decides from the geometry
 * (TdsModel.cpp:1188-1508); tests compare it bit for bit with the host restatement.  Other
 * solvers: AFS_ERR_UNSUPPORTED. */
#define AFS_PLAN_WORDS 16
/* Diagnostics: Tube::interpolate (Tube.cpp:438-505) of the pharynx/mouth areas and lengths as
 * the tree solver's synthesis kernel computes them, for n samples: frames left[n] and right[n]
 * at ratio[n] -> area[n][40], length[n][40] (host pointers).  The reference rounds each product
 * of r1 * a + ratio * b; so do the kernel and K5 (no fma contraction), which tests check bit for
 * bit.  Other solvers: AFS_ERR_UNSUPPORTED. */
afs_status afs_tube_interpolate(afs_ctx *ctx, const afs_frame *left, const afs_frame *right, const double *ratio,
                                int32_t n, double *area, double *length);
afs_status afs_noise_plans(afs_ctx *ctx, const afs_frame *frames, int32_t rows, int32_t num_frames, int32_t hop,
                           int64_t s_begin, int64_t s_end, uint64_t *plans);
/* Diagnostics: the tree solver's hop mode (hops >= AFS_PLAN_HOP_MIN): K5's hop records of the
 * hops samples [s_begin, s_end) span, hops[rows][(s_end - 1) / hop - s_begin / hop + 1]
 * [AFS_PLAN_HOP_BYTES] (layout: csrc/tree_plan.h PlanHop: per plan word its kind and inputs, the
 * mixed flag), and the dense records of the mixed hops' samples in plans (as afs_noise_plans;
 * the other samples' records are left as they were).  Host or device pointers.  Other solvers or
 * shorter hops: AFS_ERR_UNSUPPORTED. */
#define AFS_PLAN_HOP_BYTES 544
#define AFS_PLAN_HOP_MIN 32
afs_status afs_noise_plan_hops(afs_ctx *ctx, const afs_frame *frames, int32_t rows, int32_t num_frames, int32_t hop,
                               int64_t s_begin, int64_t s_end, uint8_t *hops, uint64_t *plans);
/* Diagnostics: the plan words the tree solver's synthesis kernel evaluates per sample from a hop
 * record (kernel K1's own evaluation, compiled with its flags) for n (record, ratio) pairs:
 * hops[n][AFS_PLAN_HOP_BYTES], ratio[n] -> words[n][AFS_PLAN_WORDS] (host pointers).  Outside
 * mixed hops, these words replace K5's dense records: the discrete words and sqrt(A) are the same
 * bits, the quotient words (1/A, 1/sqrt(4A/pi), the downstream factors N/D) come from a reciprocal
 * with one Newton step and a residual correction instead of an IEEE division -- within a few ulps
 * of the dense records (tests/test_plan_gpu.py measures it) -- and the downstream factors and the
 * glottis gain are hop-constant forms within 1e-12 / 1e-13 relative of the per-sample ones
 * (tests/test_plan_hops.py).  AFS_PLAN_DENSE=1 in the environment makes every hop read its dense
 * records (the per-sample plan bit for bit). */
afs_status afs_plan_hop_words(afs_ctx *ctx, const uint8_t *hops, const double *ratio, int32_t n, uint64_t *words);

/* Stateful sessions: B independent Synthesizer instances living on the device. */
afs_status afs_session_create(afs_ctx *ctx, int32_t batch, const uint32_t *seeds, afs_session **s);
/* One synthesizeSignalTds(newTube, glottisParams, num_samples, newSignal) call for every
 * utterance: frames[batch], out[batch][max(num_samples,1)].  The first call after create/reset
 * only latches the frames and produces no samples (*produced = 0). */
afs_status afs_session_synthesize(afs_session *s, const afs_frame *frames, int32_t num_samples,
                                  double *out, uint8_t *nonfinite, int32_t *produced, afs_report *report);
afs_status afs_session_reset(afs_session *s, const uint32_t *seeds);
/* rand() calls of every voice since the last reset (see afs_rng_draws). */
afs_status afs_session_rng_draws(afs_session *s, int64_t *draws);
void afs_session_destroy(afs_session *s);

/* Area-function model -> tube frames (pharynx/mouth part, teeth).  params[n][16] in
 * OneDimAreaFunction::ParamIndex order; velum and glottis fields of frames are left unchanged. */
afs_status afs_af_to_frames(afs_ctx *ctx, const double *params, int64_t n, afs_frame *frames);

/* Output format stage: out[i] = short(x * 32767) truncated towards zero, x > 1 -> 32767,
 * x < -1 -> -32768, NaN -> 0 (Synthesizer.cpp:955-973).  Host or device pointers. */
afs_status afs_to_int16(afs_ctx *ctx, const double *samples, int64_t n, int16_t *out);

/* Synthesizer::playTargetSequence(targetShape, stationary_s, transition_s)
 * (Synthesizer.cpp:1299-1422).  The reference hard-codes f0_hz {100, 115, 105, 80} (:1311), the
 * 8000 dPa lung pressure of sensorDataToGlottisParams (:903) and takes the other glottis controls
 * from TriangularGlottis' control parameters after reset() (f0 120 Hz, 10000 dPa, rest
 * displacements 0.01 cm, arytenoid area 0, aspiration -40 dB; TriangularGlottis.cpp:19-24,
 * Synthesizer.cpp:244); afs_target_sequence_default() sets those and the SURVEY config-3
 * timing (stationary 0.2/0.05/0.2/0.1 s, transitions 0.05 s). */
typedef struct afs_target_sequence {
  double stationary_s[4];
  double transition_s[3];
  double f0_hz[4];
  double lung_pressure_dpa;
  double glottis[AFS_NUM_GLOTTIS_PARAMS];  /* init() latch; [2..5] also for every sample */
} afs_target_sequence;

void afs_target_sequence_default(afs_target_sequence *ts);
/* int numSamples = SAMPLING_RATE * totalTime_s (:1328), with the context's rate. */
int64_t afs_target_sequence_samples(const afs_target_sequence *ts, double sampling_rate_hz);

/* B utterances, utterance b playing the four shapes targets[4 b .. 4 b + 3] of the shape
 * table shapes[num_shapes][16] (host pointers) with one timing for the batch.  Semantics of the
 * reference per utterance: reset + srand(seeds[b]) (NULL: b + 1), init() latches the schwa
 * tube, then one synthesizeSignalTds(tube_i, glottis_i, 1) per sample, where tube_i comes from
 * the area-function model at the cosine-interpolated parameters of sample i (teeth at xin).
 * out[B][afs_target_sequence_samples()] doubles, host or device.  Tube trajectories are built
 * on the GPU once per distinct target sequence and streamed in time chunks. */
afs_status afs_play_target_sequences(afs_ctx *ctx, const double *shapes, int32_t num_shapes,
                                     const int32_t *targets, const afs_target_sequence *ts,
                                     const uint32_t *seeds, int32_t B, double *out, uint8_t *nonfinite,
                                     afs_report *report);

/* AFS_PROFILE contexts: summed device time and count of the synthesis-kernel launches (K1), of
 * the noise-source plan launches (tree solver, K5) and of the output-stage launches (tree solver,
 * K6: glottal-tone filter, dU/dt, Chebyshev low-pass) since the previous call (waits for the
 * stream; the next call starts from zero).  afs_kernel_times is the same without K6; any pointer
 * may be NULL. */
typedef struct afs_kernel_timing {
  double synth_ms;
  int32_t synth_launches;
  double plan_ms;
  int32_t plan_launches;
  double output_ms;
  int32_t output_launches;
} afs_kernel_timing;
afs_status afs_kernel_times_ex(afs_ctx *ctx, afs_kernel_timing *timing);
afs_status afs_kernel_times(afs_ctx *ctx, double *synth_ms, int32_t *synth_launches, double *plan_ms,
                            int32_t *plan_launches);

/* ---- Several GPUs: utterance shards, the int16 audio gathered over RCCL (xGMI) ----------
 * Utterances are independent: shard r of `world` synthesizes a contiguous block with no
 * exchange; the only collective is the gather of the finished audio to rank 0.  RCCL
 * (librccl.so.1 of the ROCm installation) is loaded on first use. */
#define AFS_COMM_ID_BYTES 128 /* NCCL_UNIQUE_ID_BYTES */
typedef struct afs_comm afs_comm;

/* Block of `rank`: utterances [*first, *first + *count) of `total` over `world` ranks (the first
 * total % world ranks take one more). */
void afs_shard_range(int64_t total, int32_t world, int32_t rank, int64_t *first, int64_t *count);
/* One process per GPU: rank 0 creates the id (ncclGetUniqueId) and hands it to the other
 * ranks over any channel; every rank then joins with its context (device, stream). */
afs_status afs_comm_unique_id(uint8_t id[AFS_COMM_ID_BYTES]);
afs_status afs_comm_create(afs_ctx *ctx, const uint8_t id[AFS_COMM_ID_BYTES], int32_t rank, int32_t world,
                           afs_comm **comm);
/* One process, n GPUs: comms[i] = rank i on ctxs[i]'s device (ncclCommInitAll). */
afs_status afs_comm_create_all(afs_ctx *const *ctxs, int32_t n, afs_comm **comms);
void afs_comm_destroy(afs_comm *comm);
/* Gather `count` int16 samples (device memory of this rank's context) to rank 0's root_out
 * (device memory): rank r's block lands at the sum of the counts of ranks < r.  root_counts
 * (rank 0, world entries; NULL = every rank sends `count`).  The transfer runs on the comm's own
 * stream after the work queued so far on the context's stream, so the next synthesis overlaps
 * it; afs_comm_fence makes the context's stream wait for it (before local or root_out is
 * written again), afs_comm_synchronize waits on the host. */
afs_status afs_gather_pcm(afs_comm *comm, const int16_t *local, int64_t count, int16_t *root_out,
                          const int64_t *root_counts);
afs_status afs_comm_fence(afs_comm *comm);
afs_status afs_comm_synchronize(afs_comm *comm);
/* Device time of this rank's gathers since the previous call (HIP events on the comm's stream
 * around each afs_gather_pcm, from the moment its input is ready to the end of its sends /
 * receives) and their count; waits for the comm's stream.  Either pointer may be NULL. */
afs_status afs_comm_gather_times(afs_comm *comm, double *ms, int32_t *count);
/* The whole node from one host thread: `batch` utterances sharded over the n contexts of comms
 * (afs_comm_create_all) with afs_shard_range; each shard runs afs_synthesize on its GPU (seeds
 * keep the global index: NULL = u + 1), is converted to int16 on its GPU (afs_to_int16) and
 * gathered to ctxs[0]'s GPU.  frames[batch][num_frames] and seeds are host arrays; pcm_out
 * [batch][(num_frames-1)*hop] is host memory or device memory of ctxs[0]; nonfinite (host,
 * batch bytes) and report may be NULL.  Returns when pcm_out is complete. */
afs_status afs_multi_synthesize(afs_ctx *const *ctxs, afs_comm *const *comms, int32_t n, const afs_frame *frames,
                                const uint32_t *seeds, int32_t batch, int32_t num_frames, int32_t hop,
                                int16_t *pcm_out, uint8_t *nonfinite, afs_report *report);

#ifdef __cplusplus
}
#endif
#endif /* AFS_H */
