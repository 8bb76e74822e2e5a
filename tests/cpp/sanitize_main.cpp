// TEST-ONLY: the CPU emulator of the tree kernel (tests/emu/tree_emu.cpp over csrc/tree_core.h,
// csrc/tree_plan.h and csrc/afs_tables.cpp) and the oracle restatement (oracle/afs_oracle.c)
// in one executable built with AddressSanitizer and UndefinedBehaviorSanitizer
// (tests/test_sanitize.py).  Out-of-range LDS byte offsets in the section / step records, reads
// past the frame arrays or unintended signed overflow abort the run; the reference's own
// wrapping int sum of rand() draws (TdsModel.cpp:1690-1692) is restated with unsigned
// arithmetic, so it must not trip the overflow check.
//   sanitize_main <in> <out>
//   in:  int32 F, int32 hop, uint32 seed, double fs, int32 iopt[9], double sep_ratio, F frames
//   out: emulator samples then oracle samples ((F-1)*hop doubles each)
#include <cstdio>
#include <vector>

#include "afs_model.h"
#include "afs_oracle.h"

extern "C" long emu_tree_utterance_opt(const afs_frame *frames, int F, int hop, unsigned seed, double fs,
                                       const int *iopt, double ratio, double *out);

int main(int argc, char **argv) {
  if (argc < 3) return 2;
  FILE *fi = std::fopen(argv[1], "rb");
  if (!fi) return 3;
  int32_t F = 0, hop = 0, iopt[9];
  uint32_t seed = 1;
  double fs = 0.0, sep = 1.0;
  if (std::fread(&F, 4, 1, fi) != 1 || std::fread(&hop, 4, 1, fi) != 1 || std::fread(&seed, 4, 1, fi) != 1 ||
      std::fread(&fs, 8, 1, fi) != 1 || std::fread(iopt, 4, 9, fi) != 9 || std::fread(&sep, 8, 1, fi) != 1)
    return 3;
  if (F < 2 || hop < 1) return 3;
  std::vector<afs_frame> frames((size_t)F);
  if (std::fread(frames.data(), sizeof(afs_frame), (size_t)F, fi) != (size_t)F) return 3;
  std::fclose(fi);
  const size_t T = (size_t)(F - 1) * (size_t)hop;
  std::vector<double> emu(T), ref(T);
  if (emu_tree_utterance_opt(frames.data(), F, hop, seed, fs, iopt, sep, emu.data()) != (long)T) return 4;
  ao_options o;
  ao_default_options(&o);
  o.turbulence_losses = iopt[0];
  o.soft_walls = iopt[1];
  o.generate_noise_sources = iopt[2];
  o.radiation_from_skin = iopt[3];
  o.piriform_fossa = iopt[4];
  o.inner_length_corrections = iopt[5];
  o.transvelar_coupling = iopt[6];
  o.glottis_loss = iopt[7];
  o.glottis_model = iopt[8];
  o.flow_separation_area_ratio = sep;
  static_assert(sizeof(ao_frame) == sizeof(afs_frame), "frame layouts");
  if (ao_synthesize_utterance((const ao_frame *)frames.data(), F, hop, seed, fs, &o, ref.data()) != (long)T) return 5;
  FILE *fo = std::fopen(argv[2], "wb");
  if (!fo) return 6;
  std::fwrite(emu.data(), 8, T, fo);
  std::fwrite(ref.data(), 8, T, fo);
  std::fclose(fo);
  std::printf("ok %zu\n", T);
  return 0;
}
