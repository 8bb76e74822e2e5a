"""The tree kernel's interpolation ratio (tree_core.h hop_ratio): i * (1/hop) corrected once by the
exact remainder with an fma equals the IEEE division i / hop bit for bit -- the reference's and K5's
ratio (Tube interpolation, TdsModel / Synthesizer.cpp:515-639 driver).  Checked here for every
i < hop and every hop up to 8192, and for 2000 sampled hops up to 65536 (all their i), in C with
the C library's fma (the same operation sequence as the device code)."""
import os
import subprocess
import tempfile

SRC = r"""
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
static long check(int hop) {
  const double dhop = (double)hop, inv = 1.0 / dhop;
  long bad = 0;
  for (int i = 0; i < hop; ++i) {
    const double di = (double)i;
    volatile double q = di * inv;
    const double r = fma(-dhop, q, di);
    const double m = fma(r, inv, q);
    volatile double d = di / dhop;
    if (m != d) ++bad;
  }
  return bad;
}
int main(void) {
  long bad = 0, n = 0;
  for (int hop = 1; hop <= 8192; ++hop) { bad += check(hop); n += hop; }
  unsigned s = 12345u;
  for (int k = 0; k < 2000; ++k) {
    s = s * 1103515245u + 12345u;
    const int hop = 8193 + (int)((s >> 8) % (65536 - 8192));
    bad += check(hop); n += hop;
  }
  printf("%ld %ld\n", bad, n);
  return 0;
}
"""


def test_hop_ratio_equals_division():
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "r.c")
        exe = os.path.join(d, "r")
        open(c, "w").write(SRC)
        subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-o", exe, c, "-lm"])
        bad, n = map(int, subprocess.check_output([exe], text=True).split())
    assert n > 30_000_000
    assert bad == 0
