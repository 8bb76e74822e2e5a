"""Noise-phase variant classes of the config-4 batch and the best makespan a two-waves-per-SIMD shard
can reach (development tool, GPU box).

Each utterance's class is the lightest variant its hop records allow (tree_kernel.h noise_variant:
the or of PlanHop::noise over the launch; static vowels have the same record at every hop, so the first
hop's decides).  The slot order sorts by class inside each narrowness bucket, so waves are nearly
homogeneous.  With the measured per-variant costs (every wave forced into one variant,
profiles/r05b_noise_variant_ceiling_ab.txt: full 1, tongue-1 0.954, glottis 0.885), a SIMD's time is the
sum of its waves'; the kernel ends with the slowest SIMD.  At 16 waves per SIMD the classes average out;
at 2 the best pairing of the wave classes bounds the shard.

usage: python tools/shard_balance.py [--batch 65536] [--shard 8192]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

COST = {0: 1.0, 2: 0.954, 3: 0.885}  # NZ_FULL, NZ_TONGUE1, NZ_GLOTTIS
SERVES = {3: (1 << 48) | 0xFFFF, 2: (3 << 48) | 0xFFFFFFFF}


def classes(ctx, frames, hop, chunk=4096):
    out = []
    for r0 in range(0, frames.shape[0], chunk):
        hops, _ = ctx.noise_plan_hops(np.ascontiguousarray(frames[r0:r0 + chunk, :2]), hop, 0, hop)
        m = hops[:, :, 536:544].copy().view(np.uint64)[:, :, 0]
        m = np.bitwise_or.reduce(m, axis=1)
        c = np.zeros(m.shape, np.int64)
        c[(m & ~np.uint64(SERVES[2])) == 0] = 2
        c[(m & ~np.uint64(SERVES[3])) == 0] = 3
        out.append(c)
    return np.concatenate(out)


def best_pairing(wave_cost):
    """Makespan of the best assignment of 2 waves per SIMD: sort and pair the heaviest with the lightest."""
    w = np.sort(wave_cost)
    n = w.size // 2
    return float((w[:n] + w[::-1][:n]).max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--shard", type=int, default=8192)
    a = ap.parse_args()
    from areafunctionsynthesis_amd.synthesizer import Context
    from areafunctionsynthesis_amd.workloads import build_frames, static_vowels
    ctx = Context(44100.0, solver="tree")
    w = static_vowels(a.batch, seconds=0.02, fs=44100.0)
    frames = build_frames(w, ctx.af_to_frames)
    c = classes(ctx, frames, w.hop)
    for name, cl in (("batch", c), ("shard", c[:a.shard])):
        frac = {k: float(np.mean(cl == k)) for k in COST}
        # waves of four in class order (the slot order's class key)
        wc = np.array([max(COST[k] for k in grp) for grp in np.sort(cl)[::-1].reshape(-1, 4)])
        simds = 1024
        per_simd = wc.size / simds
        mean = float(wc.mean())
        print(f"{name}: {cl.size} utterances, classes full {frac[0]:.3f} tongue-1 {frac[2]:.3f} glottis {frac[3]:.3f}; "
              f"{wc.size} waves, {per_simd:g} per SIMD; mean wave cost {mean:.4f} (all full: 1)")
        if abs(per_simd - 2) < 1e-9:
            mk = best_pairing(wc)
            print(f"  two waves per SIMD: best pairing makespan {mk:.4f} vs the balanced {2 * mean:.4f} "
                  f"(bound on the shard's rate relative to a balanced batch: {2 * mean / mk:.4f}); all full 2.0 -> "
                  f"variant gain bound {2.0 / mk - 1:+.2%}")
        else:
            print(f"  {per_simd:g} waves per SIMD: expected time ~ mean x waves = {mean * per_simd:.3f} "
                  f"(variant gain ~{1 / mean - 1:+.2%})")
    ctx.close()


if __name__ == "__main__":
    main()
