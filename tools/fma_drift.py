"""Drift envelope of the reference itself (development tool): the C restatement compiled with
FMA contraction (-march=x86-64-v3 -ffp-contract=fast) against the reference build at -O2,
per-window max |diff| on bench.py's first 32 utterances.  Build first:
  gcc -std=c11 -O2 -march=x86-64-v3 -ffp-contract=fast -fPIC -shared -o /tmp/liboracle_fma.so oracle/afs_oracle.c -lm
"""
import sys, os, numpy as np, multiprocessing as mp
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
from oracle_lib import Oracle, RefLib
from areafunctionsynthesis_amd.workloads import static_vowels
def job(a):
    fr, seed, hop, fs = a
    x = Oracle("/tmp/liboracle_fma.so").utterance(fr, hop, seed, fs)
    y = RefLib().utterance(fr, hop, seed, fs)
    e = np.abs(x - y); edges = [0, 2048, 4410, 11025, 22050, 44100]
    return [e[a:b].max() for a, b in zip(edges[:-1], edges[1:])]
if __name__ == "__main__":
    o = Oracle()
    w = static_vowels(32, seconds=1.0, fs=44100.0)
    P = w.params
    # frames via the oracle's af restatement (same as the GPU af kernel, bit-exact by test)
    from areafunctionsynthesis_amd.workloads import build_frames
    frames = build_frames(w, lambda p: np.stack([o.af_to_frame(q) for q in p]))
    with mp.get_context("spawn").Pool(8) as pool:
        r = pool.map(job, [(frames[u], int(w.seeds[u]), w.hop, 44100.0) for u in range(32)])
    for u, v in enumerate(r): print(u, " ".join(f"{x:.1e}" for x in v))
    print("max", np.max(r, axis=0))
