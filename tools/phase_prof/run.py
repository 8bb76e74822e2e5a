"""Per-phase cycle breakdown of the tree kernel on the GPU (development tool).

python tools/phase_prof/run.py [--batch B] [--seconds S] [--workload static_vowels|fricatives]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

PHASES = ["geometry", "network", "n:filter", "n:act", "n:rng", "rows", "forward", "backward", "update",
          "output", "targets"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--seconds", type=float, default=0.05)
    ap.add_argument("--workload", default="static_vowels")
    args = ap.parse_args()
    from areafunctionsynthesis_amd import workloads
    from areafunctionsynthesis_amd.synthesizer import Context
    ctx = Context(44100.0)
    w = getattr(workloads, args.workload)(args.batch, seconds=args.seconds, fs=44100.0)
    frames = workloads.build_frames(w, ctx.af_to_frames)
    ctx.close()
    lib = ctypes.CDLL(os.path.join(HERE, os.environ.get("PP_LIB", "libphase_prof.so")))
    n = lib.pp_phase_count()
    cyc = (ctypes.c_uint64 * n)()
    ms = ctypes.c_double()
    waves = lib.pp_run(frames.ctypes.data_as(ctypes.c_void_p), w.seeds.ctypes.data_as(ctypes.c_void_p),
                       w.batch, w.num_frames, w.hop, ctypes.c_double(w.fs), cyc, ctypes.byref(ms))
    if waves <= 0:
        raise SystemExit("pp_run failed")
    T = w.samples_per_utterance
    tot = sum(cyc)
    print(f"[{os.environ.get('PP_LIB', 'libphase_prof.so')}] {args.workload} B={w.batch} T={T} waves={waves} kernel {ms.value:.2f} ms "
          f"({w.batch * T / ms.value * 1e3 / 1e6:.2f} M samples/s)")
    for p in range(n):
        print(f"  {PHASES[p]:14s} {cyc[p] / waves / T:10.1f} clk/sample  {100 * cyc[p] / tot:5.1f} %")
    print(f"  {'total':14s} {tot / waves / T:10.1f} clk/sample")
    if not hasattr(lib, "pp_wave_totals"):
        return
    wt = (ctypes.c_uint64 * waves)()
    lib.pp_wave_totals(wt)
    wt = np.array(wt, dtype=np.float64) / T
    wpb = lib.pp_waves_per_block()
    bmax = wt.reshape(-1, wpb).max(axis=1)
    print(f"  per wave: mean {wt.mean():.0f}  p10 {np.percentile(wt, 10):.0f}  p90 {np.percentile(wt, 90):.0f}  "
          f"max {wt.max():.0f};  mean of block maxima ({wpb} waves) {bmax.mean():.0f} clk/sample")


if __name__ == "__main__":
    main()
