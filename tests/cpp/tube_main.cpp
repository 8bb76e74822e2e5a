// The boundary against the reference's own Tube (src/Backend/Tube.h:14-170, compiled from
// /root/reference by oracle/Makefile into oracle/_ref/obj/Tube.o): each input frame is put into
// a real Tube through Tube::setPharynxMouthGeometry and Tube::setVelumOpening (Tube.h:130-139),
// the way the reference's callers build their tubes, and read back with
// afs::frame_from_tube<Tube> (include/afs_synthesizer.hpp).
//   tube_main <in> <out>   in: int32 F then F afs_frame records; out: F afs_frame records
// Test infrastructure only (CPU, no device calls).
#include <cstdio>
#include <vector>

#include "Tube.h"
#include "afs_synthesizer.hpp"

int main(int argc, char **argv) {
  if (argc < 3) return 2;
  FILE *fi = std::fopen(argv[1], "rb");
  if (!fi) return 3;
  int32_t F = 0;
  if (std::fread(&F, 4, 1, fi) != 1 || F <= 0) return 3;
  std::vector<afs_frame> in((size_t)F), out((size_t)F);
  if (std::fread(in.data(), sizeof(afs_frame), (size_t)F, fi) != (size_t)F) return 3;
  std::fclose(fi);
  for (int k = 0; k < F; ++k) {
    const afs_frame &f = in[(size_t)k];
    Tube::Articulator art[Tube::NUM_PHARYNX_MOUTH_SECTIONS];
    for (int i = 0; i < Tube::NUM_PHARYNX_MOUTH_SECTIONS; ++i) art[i] = (Tube::Articulator)f.articulator[i];
    Tube tube;
    tube.setPharynxMouthGeometry(f.length_cm, f.area_cm2, art, f.laterality, f.teeth_position_cm);
    tube.setVelumOpening(f.velum_opening_cm2);
    out[(size_t)k] = afs::frame_from_tube(tube, f.glottis);
  }
  FILE *fo = std::fopen(argv[2], "wb");
  if (!fo || std::fwrite(out.data(), sizeof(afs_frame), (size_t)F, fo) != (size_t)F) return 4;
  std::fclose(fo);
  std::printf("ok %d\n", F);
  return 0;
}
