/*
 * afs_synthesizer.hpp -- header-only C++ adapter for the reference's callers.
 *
 * Drops libafs (include/afs.h) in behind the reference's C++ synthesis API without touching
 * src/Backend:
 *
 *   afs::frame_from_tube(tube, glottisParams)
 *       the afs_frame of one Synthesizer::synthesizeSignalTds(Tube*, double*, int, double*)
 *       call (src/Backend/Synthesizer.h:161-162): the dynamic part of the caller's Tube
 *       (pharynxMouthSection[i].{area_cm2, length_cm, laterality, articulator},
 *       teethPosition_cm, getVelumOpening_cm2(); Tube.h:33-139) and the six
 *       TriangularGlottis control parameters.  Trachea, nose, sinus and fossa are static in
 *       the reference's Tube and the glottis sections are overwritten by the glottis model
 *       (Synthesizer.cpp:575-578), so these fields are the whole input.
 *
 *   afs::TdsVoices<TubeT>
 *       `batch` independent Synthesizer instances living on one GPU (an afs_session).
 *       synthesizeSignalTds(Tube*, double*, int, double*) has the reference's signature and
 *       semantics for batch == 1 (first call latches, n < 1 gives one sample); the array
 *       overload runs all voices in one launch.
 *
 * TubeT is the reference's Tube (or any type with the same members); the adapter has no
 * other dependency on the reference.  Errors throw afs::Error with afs_last_error().
 */
#ifndef AFS_SYNTHESIZER_HPP
#define AFS_SYNTHESIZER_HPP

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "afs.h"

namespace afs {

struct Error : std::runtime_error {
  afs_status status;
  Error(afs_status s, const std::string &what) : std::runtime_error(what), status(s) {}
};

inline void check(afs_status s, const afs_ctx *ctx, const char *call) {
  if (s == AFS_OK) return;
  std::string msg = std::string(call) + ": " + afs_status_string(s);
  if (ctx) {
    const char *e = afs_last_error(ctx);
    if (e && *e) msg += std::string(" (") + e + ")";
  }
  throw Error(s, msg);
}

template <class TubeT>
inline afs_frame frame_from_tube(const TubeT &tube, const double *glottisParams) {
  afs_frame f;
  std::memset(&f, 0, sizeof f);
  for (int i = 0; i < AFS_NUM_TUBE_SECTIONS; ++i) {
    const auto &s = tube.pharynxMouthSection[i];
    f.area_cm2[i] = s.area_cm2;
    f.length_cm[i] = s.length_cm;
    f.laterality[i] = s.laterality;
    f.articulator[i] = (uint8_t)s.articulator;
  }
  f.teeth_position_cm = tube.teethPosition_cm;
  f.velum_opening_cm2 = tube.getVelumOpening_cm2();
  for (int k = 0; k < AFS_NUM_GLOTTIS_PARAMS; ++k) f.glottis[k] = glottisParams[k];
  return f;
}

// One GPU context (device, sampling rate, TdsModel options) shared by sessions.
class Context {
 public:
  explicit Context(double sampling_rate_hz = 22050.0, int device = 0) {
    afs_config cfg;
    afs_config_default(&cfg);
    cfg.sampling_rate_hz = sampling_rate_hz;
    cfg.device = device;
    check(afs_create(&ctx_, &cfg), nullptr, "afs_create");
  }
  explicit Context(const afs_config &cfg) { check(afs_create(&ctx_, &cfg), nullptr, "afs_create"); }
  ~Context() { afs_destroy(ctx_); }
  Context(const Context &) = delete;
  Context &operator=(const Context &) = delete;
  afs_ctx *get() const { return ctx_; }

 private:
  afs_ctx *ctx_ = nullptr;
};

template <class TubeT>
class TdsVoices {
 public:
  // seeds: srand() seed per voice (nullptr: 1, 2, ..., batch)
  TdsVoices(Context &ctx, int batch = 1, const uint32_t *seeds = nullptr) : ctx_(ctx), batch_(batch) {
    check(afs_session_create(ctx.get(), batch, seeds, &s_), ctx.get(), "afs_session_create");
    frames_.resize((size_t)batch);
  }
  ~TdsVoices() { afs_session_destroy(s_); }
  TdsVoices(const TdsVoices &) = delete;
  TdsVoices &operator=(const TdsVoices &) = delete;

  // Synthesizer::reset + srand(seed) for every voice.
  void reset(const uint32_t *seeds = nullptr) { check(afs_session_reset(s_, seeds), ctx_.get(), "afs_session_reset"); }

  // Synthesizer::synthesizeSignalTds for voice 0 (batch == 1).  Returns the number of
  // samples written (0 for the latching first call).
  int synthesizeSignalTds(const TubeT *newTube, const double *newGlottisParams, int numNewSamples,
                          double *newSignal) {
    if (batch_ != 1) throw Error(AFS_ERR_INVALID_ARGUMENT, "single-voice call on a batched TdsVoices");
    return synthesizeSignalTds(&newTube, &newGlottisParams, numNewSamples, &newSignal);
  }

  // All voices at once: tubes[b], glottisParams[b], newSignals[b] (each >= max(n, 1) doubles).
  int synthesizeSignalTds(const TubeT *const *newTubes, const double *const *newGlottisParams,
                          int numNewSamples, double *const *newSignals) {
    for (int b = 0; b < batch_; ++b) frames_[(size_t)b] = frame_from_tube(*newTubes[b], newGlottisParams[b]);
    const int n = numNewSamples < 1 ? 1 : numNewSamples;
    out_.resize((size_t)batch_ * (size_t)n);
    int32_t produced = 0;
    check(afs_session_synthesize(s_, frames_.data(), numNewSamples, out_.data(), nullptr, &produced, nullptr), ctx_.get(),
          "afs_session_synthesize");
    for (int b = 0; b < batch_; ++b)
      if (newSignals[b] && produced > 0)
        std::memcpy(newSignals[b], out_.data() + (size_t)b * (size_t)n, sizeof(double) * (size_t)produced);
    return produced;
  }

  int batch() const { return batch_; }

 private:
  Context &ctx_;
  int batch_;
  afs_session *s_ = nullptr;
  std::vector<afs_frame> frames_;
  std::vector<double> out_;
};

}  // namespace afs

#endif  // AFS_SYNTHESIZER_HPP
