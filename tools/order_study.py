"""Study (development tool, GPU): does the order of the utterances in a batch change the synthesis
kernel's time?  A wave runs four utterances in lockstep, so it pays for the union of their
branches (noise sources that need the exponential of a cutoff, mixed hops), and the launch ends
with its slowest compute unit.  Times afs_synthesize on the config-4 static-vowel shard in the
generator's order and sorted by the vowel each utterance plays (identical audio per utterance),
alternating.

python tools/order_study.py [--batch 8192] [--seconds 1.0] [--reps 3] [--workload static_vowels]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--seconds", type=float, default=1.0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--workload", default="static_vowels", choices=("static_vowels", "fricatives"))
    args = ap.parse_args()
    import torch
    from areafunctionsynthesis_amd import workloads
    from areafunctionsynthesis_amd.frames import FRAME_DTYPE
    from areafunctionsynthesis_amd.synthesizer import Context

    B = args.batch
    ctx = Context(44100.0, solver="tree", profile=True)
    gen = getattr(workloads, args.workload)
    w = gen(B, seconds=args.seconds, fs=44100.0)
    frames = workloads.build_frames(w, ctx.af_to_frames)
    seed = workloads.BUILD_SEED + (5 if args.workload == "fricatives" else 0)
    n = len(workloads.VOWELS if args.workload == "static_vowels" else workloads.FRICATIVES)
    pick, _, uni = workloads._rows(seed, 0, B, n)
    orders = {"generator": np.arange(B), "by_shape": np.lexsort((uni[:, 0], pick))}
    seeds = np.asarray(w.seeds, dtype=np.uint32)
    dev = torch.device("cuda", 0)
    inputs = {}
    for name, o in orders.items():
        fr = np.ascontiguousarray(frames[o])
        inputs[name] = (torch.from_numpy(fr.view(np.uint8).reshape(B, w.num_frames, FRAME_DTYPE.itemsize)).to(dev),
                        torch.from_numpy(seeds[o].copy()).to(dev))
    out = torch.empty((B, w.samples_per_utterance), dtype=torch.float64, device=dev)
    ref = {}
    for name, (f, s) in inputs.items():  # warm-up, and the audio of each order
        ctx.synthesize(f, w.hop, seeds=s, out=out)
        torch.cuda.synchronize()
        ref[name] = out[:8].cpu().numpy().copy() if name == "generator" else None
        ctx.kernel_times()
    # the sorted batch's rows are the generator's rows permuted: check a few
    o = orders["by_shape"]
    f, s = inputs["by_shape"]
    ctx.synthesize(f, w.hop, seeds=s, out=out)
    torch.cuda.synchronize()
    ctx.kernel_times()
    inv = np.argsort(o)
    got = out[torch.from_numpy(inv[:8]).to(dev)].cpu().numpy()
    print("sorted rows equal the generator's rows bit for bit:", bool(np.array_equal(got, ref["generator"])), flush=True)
    for rep in range(args.reps):
        for name, (f, s) in inputs.items():
            ctx.synthesize(f, w.hop, seeds=s, out=out)
            torch.cuda.synchronize()
            kt = ctx.kernel_times()
            print(f"rep {rep} {name:10s} K1 {kt['synth_ms']:.2f} ms in {kt['synth_launches']} launches, "
                  f"K5 {kt['plan_ms']:.2f} ms, K6 {kt['output_ms']:.2f} ms", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
