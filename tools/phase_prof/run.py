"""Per-phase cycle breakdown of the tree kernel on the GPU (development tool).

python tools/phase_prof/run.py [--batch B] [--seconds S] [--workload static_vowels|fricatives]
(PP_HOPS=1: K5's hop records and the noise-phase variants, as large calls run; PP_PAIR_ROLES=1: the
wave-pair build's phases by role and its SIMD placement)
"""
import argparse
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

PHASES = ["geometry", "network", "n:filter", "n:act", "n:rng", "rows", "forward", "backward", "update",
          "output", "targets", "pair:P1 wait", "pair:P2 wait", "pair:P3 wait", "pair:P4 wait", "pair:rng (DYN)",
          "pair:tail", "pair:glottis+static net (STAT)", "pair:targets (STAT)", "pair:interp+glottis (DYN)",
          "pair:P0 wait", "(placement)", "(t0)", "(t1)"]
PLACE = 21  # tree_core.h PH_PLACE_HW, then the loop's first and last memtime


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
    if os.environ.get("PP_HOPS"):  # (hop records, noise-phase variants, slots ordered by noise class)
        lib.pp_set_hops(1)
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
        if cyc[p]:
            print(f"  {PHASES[p]:14s} {cyc[p] / waves / T:10.1f} clk/sample  {100 * cyc[p] / tot:5.1f} %")
    print(f"  {'total':14s} {tot / waves / T:10.1f} clk/sample")
    if not hasattr(lib, "pp_wave_totals"):
        return
    if os.environ.get("PP_PAIR_ROLES"):  # (wave-pair builds: a wave is DYN when it timed a network phase)
        per = (ctypes.c_uint64 * (waves * n))()
        lib.pp_wave_phases(per)
        raw = np.array(per, dtype=np.uint64).reshape(waves, n)
        hw, t0, t1 = raw[:, PLACE].copy(), raw[:, PLACE + 1].astype(np.int64), raw[:, PLACE + 2].astype(np.int64)
        a = raw.astype(np.float64)
        a[:, PLACE:PLACE + 3] = 0
        dyn = a[:, 1] > 0
        for role, m in (("DYN", dyn), ("STAT", ~dyn)):
            r = a[m].sum(axis=0) / max(1, m.sum()) / T
            print(f"  {role} ({m.sum()} waves): " + ", ".join(f"{PHASES[p]} {r[p]:.0f}" for p in range(n) if r[p] > 0.5) +
                  f"; total {r.sum():.0f} clk/sample")
        # placement: SIMD of each wave, the CU (XCC, SE, SH, CU) of each workgroup; waves that share a SIMD
        # while both run, by their roles (weighted by the overlap of their loops' spans)
        simd = (hw >> np.uint64(4)) & np.uint64(3)
        cu = ((hw >> np.uint64(32)) << np.uint64(8)) | ((hw >> np.uint64(8)) & np.uint64(255))
        wpb = lib.pp_waves_per_block()
        blk = np.arange(waves) // wpb
        spread = np.mean([len(set(simd[b * wpb:(b + 1) * wpb].tolist())) == wpb for b in range(waves // wpb)])
        pairs = {"DYN+DYN": 0.0, "DYN+STAT": 0.0, "STAT+STAT": 0.0}
        key = (cu << np.uint64(2)) | simd
        order = np.argsort(key, kind="stable")
        ks = key[order]
        bounds = np.flatnonzero(np.diff(ks.astype(np.int64))) + 1
        for grp in np.split(order, bounds):
            for x in range(len(grp)):
                for y in range(x + 1, len(grp)):
                    i, j = grp[x], grp[y]
                    if blk[i] == blk[j]:
                        continue
                    ov = min(t1[i], t1[j]) - max(t0[i], t0[j])
                    if ov > 0:
                        pairs[["STAT+STAT", "DYN+STAT", "DYN+DYN"][int(dyn[i]) + int(dyn[j])]] += ov
        tot_ov = sum(pairs.values()) or 1.0
        xcc = sorted(set((hw >> np.uint64(32)).tolist()))
        print(f"  placement: workgroups on {wpb} distinct SIMDs {100 * spread:.1f} %; XCC ids {xcc}; SIMD sharing by roles " +
              ", ".join(f"{k} {100 * v / tot_ov:.1f} %" for k, v in pairs.items()))
    wt = (ctypes.c_uint64 * waves)()
    lib.pp_wave_totals(wt)
    wt = np.array(wt, dtype=np.float64) / T
    wpb = lib.pp_waves_per_block()
    bmax = wt.reshape(-1, wpb).max(axis=1)
    print(f"  per wave: mean {wt.mean():.0f}  p10 {np.percentile(wt, 10):.0f}  p90 {np.percentile(wt, 90):.0f}  "
          f"max {wt.max():.0f};  mean of block maxima ({wpb} waves) {bmax.mean():.0f} clk/sample")


if __name__ == "__main__":
    main()
