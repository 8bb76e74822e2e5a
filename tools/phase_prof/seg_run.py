"""Per-phase cycle breakdown of the seg kernel on the GPU (development tool).

python tools/phase_prof/seg_run.py [--batch B] [--seconds S] [--workload static_vowels|fricatives]
"""
import argparse
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

PHASES = ["(loop) + block 1", "noise", "rows", "solve", "update + output", "-", "-", "-"]


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
    lib = ctypes.CDLL(os.path.join(HERE, os.environ.get("SP_LIB", "libseg_prof.so")))
    n = lib.sp_phase_count()
    cyc = (ctypes.c_uint64 * n)()
    ms = ctypes.c_double()
    waves = lib.sp_run(frames.ctypes.data_as(ctypes.c_void_p), w.seeds.ctypes.data_as(ctypes.c_void_p),
                       w.batch, w.num_frames, w.hop, ctypes.c_double(w.fs), cyc, ctypes.byref(ms))
    if waves <= 0:
        raise SystemExit("sp_run failed")
    T = w.samples_per_utterance
    tot = sum(cyc)
    print(f"[seg] {args.workload} B={w.batch} T={T} waves={waves} kernel {ms.value:.2f} ms "
          f"({w.batch * T / ms.value * 1e3 / 1e6:.2f} M samples/s)")
    for p in range(n):
        if cyc[p]:
            print(f"  {PHASES[p]:18s} {cyc[p] / waves / T:10.1f} clk/sample  {100 * cyc[p] / tot:5.1f} %")
    print(f"  {'total':18s} {tot / waves / T:10.1f} clk/sample")


if __name__ == "__main__":
    main()
