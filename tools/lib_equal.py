"""Bitwise comparison of two builds' audio (development tool, GPU box): synthesizes the same batches
with the library this process loads (AFS_LIB) and writes them to an .npz, or compares two such files.

usage: AFS_LIB=.../libafs_A.so python tools/lib_equal.py write out_A.npz
       python tools/lib_equal.py compare out_A.npz out_B.npz
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def write(path):
    from areafunctionsynthesis_amd import workloads
    from areafunctionsynthesis_amd.synthesizer import Context, Synthesizer as Session
    out = {}
    for fs in (44100.0, 22050.0):
        lanes = int(os.environ.get("AFS_EQ_LANES", "0")) or None  # (16: the throughput kernel at this small batch)
        ctx = Context(fs, solver="tree", lanes=lanes)
        for name, gen in (("static", workloads.static_vowels), ("fricatives", workloads.fricatives)):
            w = gen(96, seconds=0.3, fs=fs)
            frames = workloads.build_frames(w, ctx.af_to_frames)
            out[f"{name}_{fs:g}"] = ctx.synthesize(frames, w.hop, seeds=w.seeds)
            out[f"{name}_{fs:g}_draws"] = ctx.rng_draws(w.batch)
            # a session of 1102-sample calls over the first utterances (the window flushes at call ends)
            s = Session(ctx, batch=4, seeds=w.seeds[:4])
            ys = [s.synthesize_signal_tds(np.ascontiguousarray(frames[:4, k]), 1102 if k else 0)
                  for k in range(frames.shape[1])]
            out[f"{name}_{fs:g}_session"] = np.concatenate([y for y in ys if y is not None and y.size], axis=1)
            s.close()
        ctx.close()
    np.savez(path, **out)


def compare(a, b):
    A, Bz = np.load(a), np.load(b)
    bad = 0
    for k in A.files:
        same = np.array_equal(A[k], Bz[k])
        d = float(np.abs(A[k].astype(np.float64) - Bz[k].astype(np.float64)).max())
        print(f"{k:28s} bitwise {same}  max|diff| {d:.3e}")
        bad += not same
    print("ALL EQUAL" if not bad else f"{bad} DIFFER")
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "write":
        write(sys.argv[2])
    else:
        sys.exit(1 if compare(sys.argv[2], sys.argv[3]) else 0)
