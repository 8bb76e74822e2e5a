"""fp32 tube state: how far is it from the fp64 reference?  (BASELINE config 3 names an fp32
tube state; the north star bounds the per-utterance RMS error at 1e-4.)

python tools/fp32_study/study.py [--workload static_vowels|fricatives] [--n 6] [--seconds 1]

Runs the fp64 oracle restatement (pinned bit-exact against the reference build) and its fp32
variant (tools/fp32_study/build.sh) on the same frames and seeds, and prints the signal RMS,
the error RMS per utterance and per quarter of the utterance.
"""
import argparse
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="static_vowels")
    ap.add_argument("--n", type=int, default=6)
    ap.add_argument("--seconds", type=float, default=1.0)
    a = ap.parse_args()
    lib = subprocess.check_output([os.path.join(HERE, "build.sh")], text=True).strip().splitlines()[-1]
    from oracle_lib import Oracle
    from areafunctionsynthesis_amd import workloads
    o64, o32 = Oracle(), Oracle(lib)
    w = getattr(workloads, a.workload)(a.n, seconds=a.seconds, fs=44100.0)
    frames = workloads.build_frames(w, lambda P: np.stack([o64.af_to_frame(p) for p in P]))
    worst = 0.0
    for u in range(a.n):
        x = o64.utterance(frames[u], w.hop, int(w.seeds[u]), w.fs)
        y = o32.utterance(frames[u], w.hop, int(w.seeds[u]), w.fs)
        e = y - x
        q = len(x) // 4
        rms = float(np.sqrt(np.mean(e * e)))
        worst = max(worst, rms)
        quarters = " ".join(f"{np.sqrt(np.mean(e[i * q:(i + 1) * q] ** 2)):.1e}" for i in range(4))
        print(f"{a.workload} u{u}: signal RMS {np.sqrt(np.mean(x * x)):.3e}  error RMS {rms:.3e}  "
              f"max |err| {np.abs(e).max():.3e}  per-quarter RMS {quarters}")
    print(f"worst per-utterance RMS {worst:.3e} vs the north-star bound 1e-4 ({worst / 1e-4:.0f}x)")


if __name__ == "__main__":
    main()
