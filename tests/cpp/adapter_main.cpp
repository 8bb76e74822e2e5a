// Test driver for include/afs_synthesizer.hpp.  MockTube has the members the adapter reads,
// with the reference's names and types (Tube.h:33-139); no reference code is used.
//   adapter_main frames <file>        print afs_frame fields of a mock tube (CPU)
//   adapter_main nodevice             create a context on a missing device -> afs::Error (CPU)
//   adapter_main synth <in> <out>     run TdsVoices (batch 1) over frames read from <in> (GPU)
//   adapter_main latency <in> <out>   the same, writing per call (ms): wall time, tube conversion,
//                                     K5, K1, K6 device times (AFS_PROFILE events) to <out>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "afs_synthesizer.hpp"

struct MockTube {
  enum Articulator { VOCAL_FOLDS, TONGUE, LOWER_INCISORS, LOWER_LIP, OTHER_ARTICULATOR, NUM_ARTICULATORS };
  struct Section {
    double pos_cm, area_cm2, length_cm, volume_cm3, wallMass_cgs, wallStiffness_cgs, wallResistance_cgs;
    Articulator articulator;
    double laterality;
  };
  Section pharynxMouthSection[40];
  Section noseSection[19];
  double teethPosition_cm;
  double aspirationStrength_dB;
  double getVelumOpening_cm2() const { return noseSection[0].area_cm2; }
};

static void fill(MockTube &t, const afs_frame &f) {
  std::memset(&t, 0, sizeof t);
  for (int i = 0; i < 40; ++i) {
    t.pharynxMouthSection[i].area_cm2 = f.area_cm2[i];
    t.pharynxMouthSection[i].length_cm = f.length_cm[i];
    t.pharynxMouthSection[i].laterality = f.laterality[i];
    t.pharynxMouthSection[i].articulator = (MockTube::Articulator)f.articulator[i];
  }
  t.teethPosition_cm = f.teeth_position_cm;
  t.noseSection[0].area_cm2 = f.velum_opening_cm2;
}

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  if (!std::strcmp(argv[1], "frames")) {
    // round trip: frame -> MockTube -> frame_from_tube -> frame, bytes must match
    afs_frame f;
    std::memset(&f, 0, sizeof f);
    for (int i = 0; i < 40; ++i) {
      f.area_cm2[i] = 0.5 + 0.01 * i;
      f.length_cm[i] = 0.4 + 0.001 * i;
      f.laterality[i] = (i % 7) * 0.1;
      f.articulator[i] = (uint8_t)(i % 5);
    }
    f.teeth_position_cm = 15.25;
    f.velum_opening_cm2 = 0.75;
    const double gp[6] = {120.0, 8000.0, 0.01, 0.02, 0.03, -40.0};
    for (int k = 0; k < 6; ++k) f.glottis[k] = gp[k];
    MockTube t;
    fill(t, f);
    afs_frame g = afs::frame_from_tube(t, gp);
    std::printf("%s\n", std::memcmp(&f, &g, sizeof f) == 0 ? "frames-equal" : "frames-differ");
    return 0;
  }
  if (!std::strcmp(argv[1], "nodevice")) {
    try {
      afs::Context ctx(22050.0, 4096);
      std::printf("no-error\n");
    } catch (const afs::Error &e) {
      std::printf("error %d\n", (int)e.status);
    }
    return 0;
  }
  const bool latency = !std::strcmp(argv[1], "latency");
  if ((!std::strcmp(argv[1], "synth") || latency) && argc >= 5) {
    // <in>: int32 F, int32 hop, double fs, uint32 seed, then F afs_frame records
    FILE *fi = std::fopen(argv[2], "rb");
    if (!fi) return 3;
    int32_t F = 0, hop = 0;
    double fs = 0;
    uint32_t seed = 1;
    if (std::fread(&F, 4, 1, fi) != 1 || std::fread(&hop, 4, 1, fi) != 1 || std::fread(&fs, 8, 1, fi) != 1 ||
        std::fread(&seed, 4, 1, fi) != 1)
      return 3;
    std::vector<afs_frame> fr((size_t)F);
    if (std::fread(fr.data(), sizeof(afs_frame), (size_t)F, fi) != (size_t)F) return 3;
    std::fclose(fi);
    (void)argv[4];
    afs_config cfg;
    afs_config_default(&cfg);
    cfg.sampling_rate_hz = fs;
    if (latency) cfg.flags |= AFS_PROFILE;  // (per-call kernel times, read after each call's clock)
    afs::Context ctx(cfg);
    afs::TdsVoices<MockTube> voice(ctx, 1, &seed);
    std::vector<double> out, ms;
    std::vector<double> buf((size_t)hop);
    using clk = std::chrono::steady_clock;
    auto msec = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    for (int k = 0; k < F; ++k) {
      MockTube t;
      fill(t, fr[(size_t)k]);
      // the host's tube conversion alone (the call below repeats it)
      const auto c0 = clk::now();
      volatile afs_frame probe = afs::frame_from_tube(t, fr[(size_t)k].glottis);
      (void)probe;
      const auto c1 = clk::now();
      // (one call as SynthesisThread makes it: tube + glottis in, hop samples back in host memory)
      const auto t0 = clk::now();
      int n = voice.synthesizeSignalTds(&t, fr[(size_t)k].glottis, hop, buf.data());
      const auto t1 = clk::now();
      if (latency) {
        // per call: wall, tube conversion, K5, K1, K6 device times (HIP events around each launch)
        afs_kernel_timing kt{};
        afs::check(afs_kernel_times_ex(ctx.get(), &kt), ctx.get(), "afs_kernel_times_ex");
        for (double v : {msec(t0, t1), msec(c0, c1), kt.plan_ms, kt.synth_ms, kt.output_ms}) ms.push_back(v);
      }
      out.insert(out.end(), buf.begin(), buf.begin() + n);
    }
    if (latency) out = ms;
    FILE *fo = std::fopen(argv[3], "wb");
    std::fwrite(out.data(), sizeof(double), out.size(), fo);
    std::fclose(fo);
    std::printf("samples %zu\n", out.size());
    return 0;
  }
  return 2;
}
