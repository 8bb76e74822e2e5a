"""Benchmark: batched time-domain tube synthesis on MI355X.

python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--seconds S] [--fs HZ]
For N > 1 launch with torch.distributed.run (one rank per GPU, RCCL).

One *step* = one pass of the hot path over this rank's shard of the BASELINE config-4
batch: B static-vowel utterances (default 8192 per GPU; 65536 at 8 GPUs) of S seconds at
fs Hz, from frames already resident in HBM to fp64 audio in HBM, converted on the GPU to
the reference's int16 output format and (N > 1) gathered to rank 0 over RCCL while the next
step synthesizes.  Scaling is weak: per-GPU work is fixed.

Printed (rank 0): one JSON line with the BASELINE metric (whole-node samples/s), the
roofline object of the dominant kernel and the CPU baseline (the reference's own
sources, oracle/_ref, timed on this host's cores over a bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md, chip-level parameters (spec)
FP64_PEAK_TFLOPS = 78.6        # MI355X FP64 vector peak (spec)
# fp64 lane-flops per utterance-sample executed by the tree kernel, counted on the GPU:
# SQ_INSTS_VALU_FLOPS_FP64 counts flops per wave-instruction (2050.3 per wave-sample), x 64 lanes
# / 4 utterances per wave (profiles/r01_pmc_sq_v2p.txt).  Lane-uniform work (glottis, output
# stage) is counted on every lane.  (SURVEY.md 8(a)'s 1.8e4 is the reference algorithm's count.)
FLOPS_PER_SAMPLE = 32805.0


def pmc_traffic(kernel: str, workload: str, batch: int, samples: int, hop: int):
    """HBM bytes per launch of `kernel` from the committed PMC passes (profiles/pmc_traffic.json,
    written by tools/pmc_traffic.py from rocprofv3 FETCH_SIZE / WRITE_SIZE runs of this same
    command), or None when no pass covers this configuration."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None, None
    e = json.load(open(path)).get(f"{kernel}|{workload}|B={batch}|T={samples}|hop={hop}")
    return (e["traffic_bytes_per_launch"], e["tag"]) if e else (None, None)


def frame_bytes_per_sample(hop: int) -> float:
    # one 1072-B frame per hop samples + one 8-B fp64 output sample
    return 1072.0 / hop + 8.0


def cpu_baseline(jobs, fs: float, n_utt: int, gpu_out: np.ndarray, what: str):
    """Time the reference build (oracle/_ref) on a bounded sample, one process per core.
    jobs[u] = ("frames", frames, seed, hop) or ("target", shapes4, seed, None)."""
    import multiprocessing as mp

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import REF_SO, ORACLE_SO  # noqa: F401

    kind = "reference" if os.path.exists(REF_SO) else "port"
    cores = max(1, min(16, os.cpu_count() or 1, n_utt))
    jobs = [(kind,) + tuple(j) + (fs,) for j in jobs]
    ctx = mp.get_context("spawn")
    t0 = time.perf_counter()
    with ctx.Pool(cores) as pool:
        outs = pool.map(_cpu_job, jobs)
    wall = time.perf_counter() - t0
    samples = sum(o.size for o in outs)
    errs = [float(np.abs(gpu_out[u] - outs[u]).max()) for u in range(n_utt)]
    rmss = [float(np.sqrt(np.mean((gpu_out[u] - outs[u]) ** 2))) for u in range(n_utt)]
    return {
        "value": samples / wall,
        "unit": "samples/s",
        "cores": cores,
        "kind": kind,
        "sample": f"{n_utt} utterances ({what}) @ {fs:g} Hz (first utterances of this shard), {cores} processes",
        "wall_s": wall,
    }, max(errs), max(rmss)


def _cpu_job(job):
    kind, what, data, seed, hop, fs = job
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import Oracle, RefLib
    lib = RefLib() if kind == "reference" else Oracle()
    if what == "target":  # playTargetSequence: per-sample area function -> tube, then n = 1 calls
        return lib.utterance(Oracle().target_frames(data, fs), 1, seed, fs)
    return lib.utterance(data, hop, seed, fs)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=8192, help="utterances per GPU")
    ap.add_argument("--seconds", type=float, default=1.0)
    ap.add_argument("--fs", type=float, default=44100.0)
    ap.add_argument("--solver", default=os.environ.get("AFS_SOLVER", "tree"))
    ap.add_argument("--cpu-utterances", type=int, default=32)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", choices=("static", "vcv"), default="static",
                    help="static: config-4 shard of static vowels (default); vcv: config-3 VCV "
                         "utterances through playTargetSequence (per-sample tubes, hop 1)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from areafunctionsynthesis_amd import sharding
    from areafunctionsynthesis_amd.frames import FRAME_DTYPE
    from areafunctionsynthesis_amd.synthesizer import Context
    from areafunctionsynthesis_amd.workloads import build_frames, static_vowels, vcv_targets

    B = args.batch
    ctx = Context(args.fs, solver=args.solver, device=local, async_calls=True)
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)

    first, _ = sharding.shard_range(rank, world, B)
    max_launch_samples = 65536 if args.solver == "tree" else 8192
    if args.workload == "static":
        w = static_vowels(B, seconds=args.seconds, fs=args.fs, first_utterance=first)
        frames = build_frames(w, ctx.af_to_frames)
        F, hop, T = w.num_frames, w.hop, w.samples_per_utterance
        seeds = w.seeds
        frames_dev = torch.from_numpy(frames.view(np.uint8).reshape(B, F, FRAME_DTYPE.itemsize)).to(dev)
        launches_per_step = -(-(F - 1) // max(1, max_launch_samples // hop))

        def synth():
            ctx.synthesize(frames_dev, hop, seeds=seeds_dev, out=out_dev)
    else:
        shapes, targets, seeds = vcv_targets(B, first_utterance=first)
        hop, T = 1, ctx.target_sequence_samples()
        launches_per_step = -(-T // max_launch_samples)

        def synth():
            ctx.play_target_sequences(shapes, targets, seeds=seeds_dev, out=out_dev)
    seeds_dev = torch.from_numpy(seeds.astype(np.int32)).to(dev)
    out_dev = torch.empty((B, T), dtype=torch.float64, device=dev)

    # the reference's output format (int16, Synthesizer.cpp:955-973) is produced on the GPU
    # and gathered to rank 0 while the next step synthesizes
    pcm = sharding.PcmGather(lambda x, o: ctx.to_int16(x, out=o), (B, T), world, rank, dist, device=dev)

    def step():
        synth()
        pcm.submit(out_dev)

    for _ in range(args.warmup):
        step()
    pcm.drain()
    torch.cuda.synchronize(dev)

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        synth()
        ev[k][1].record(stream)
        pcm.submit(out_dev)
    pcm.drain()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    synth_ms = [a.elapsed_time(b) for a, b in ev]
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    if rank == 0:
        total_samples = float(world) * B * T * args.steps
        value = total_samples / elapsed
        ms_step = elapsed / args.steps * 1e3
        avg_launch_s = (np.mean(synth_ms) / 1e3) / launches_per_step
        samples_per_launch = B * T / launches_per_step
        alg_bytes = samples_per_launch * frame_bytes_per_sample(hop)
        achieved_gbs = alg_bytes / avg_launch_s / 1e9
        flops = samples_per_launch * FLOPS_PER_SAMPLE
        kname = "lane_synth_kernel" if args.solver == "cholesky" else "tree_synth_kernel"
        traffic, traffic_tag = (None, None)
        if launches_per_step == 1:
            traffic, traffic_tag = pmc_traffic(kname, args.workload, B, T, hop)
        result = {
            "metric": "audio samples/s (whole node) on 64k-utterance batch; max-abs err vs CPU ref",
            "value": value,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": (f"BASELINE config 4 shard: {B} static-vowel utterances/GPU x {args.seconds:g} s "
                             f"@ {args.fs:g} Hz ({B * 8} at 8 GPUs), frames resident in HBM")
                if args.workload == "static" else
                (f"BASELINE config 3 (fp64 state): {B} VCV utterances/GPU through playTargetSequence "
                 f"({T} samples @ {args.fs:g} Hz, per-sample area-function tubes built on the GPU)"),
                "batch_per_gpu": B,
                "global_batch": B * world,
                "samples_per_utterance": T,
                "fs_hz": args.fs,
                "hop": hop,
                "solver": args.solver,
                "parallelism": f"dp{world} (utterance shards, int16 audio gathered to rank 0 over RCCL, overlapped)" if world > 1
                               else "dp1",
            },
            "x_realtime": value / args.fs,
            "roofline": {
                "bound": "hbm",
                "achieved": achieved_gbs,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved_gbs / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_unit": "bytes per launch (rocprofv3 PMC: 2 x FETCH_SIZE + WRITE_SIZE, gfx950-corrected)",
                "traffic_source": f"profiles/pmc_traffic.json [{traffic_tag}]" if traffic else None,
                "algorithmic_bytes_per_launch": alg_bytes,
                "kernel": kname,
                "avg_launch_ms": avg_launch_s * 1e3,
                "launches_per_step": launches_per_step,
                "bytes_per_sample": frame_bytes_per_sample(hop),
                "fp64_achieved_tflops": flops / avg_launch_s / 1e12,
                "fp64_peak_tflops": FP64_PEAK_TFLOPS,
            },
        }
        if world == 1 and not args.no_cpu_baseline:
            n = min(args.cpu_utterances, B)
            gpu_out = out_dev[:n].cpu().numpy()
            if args.workload == "static":
                jobs = [("frames", frames[u], int(seeds[u]), hop) for u in range(n)]
                what = f"{F - 1} frames x {hop} samples"
            else:
                jobs = [("target", shapes[targets[u]], int(seeds[u]), None) for u in range(n)]
                what = f"playTargetSequence, {T} samples, trajectory built per sample on the CPU"
            cb, max_abs, max_rms = cpu_baseline(jobs, args.fs, n, gpu_out, what)
            cb.pop("wall_s")
            result["cpu_baseline"] = cb
            result["max_abs_err_vs_cpu_ref"] = max_abs
            result["max_rms_err_vs_cpu_ref"] = max_rms
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
