"""Error growth of the GPU output against the reference build over a long utterance
(development tool): bench.py's workload rows, per-window max |gpu - ref|."""
import multiprocessing as mp
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _ref(job):
    from oracle_lib import RefLib
    fr, seed, hop, fs = job
    return RefLib().utterance(fr, hop, seed, fs)


def main():
    from areafunctionsynthesis_amd import _native
    if len(sys.argv) > 1:
        _native.load(sys.argv[1])
    from areafunctionsynthesis_amd.synthesizer import Context
    from areafunctionsynthesis_amd.workloads import build_frames, static_vowels
    n, fs = int(os.environ.get("DRIFT_N", "32")), 44100.0
    ctx = Context(fs)
    w = static_vowels(n, seconds=1.0, fs=fs)
    frames = build_frames(w, ctx.af_to_frames)
    y = ctx.synthesize(frames, w.hop, seeds=w.seeds)
    with mp.get_context("spawn").Pool(16) as pool:
        refs = pool.map(_ref, [(frames[u], int(w.seeds[u]), w.hop, fs) for u in range(n)])
    edges = [0, 2048, 4410, 11025, 22050, 44100]
    for u in range(n):
        e = np.abs(y[u] - refs[u])
        win = [e[a:b].max() for a, b in zip(edges[:-1], edges[1:])]
        print(f"utt {u:3d} seed {int(w.seeds[u]):3d} " + " ".join(f"{v:.1e}" for v in win)
              + f"  peak|y| {np.abs(refs[u]).max():.2e}")


if __name__ == "__main__":
    main()
