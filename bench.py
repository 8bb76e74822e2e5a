"""Benchmark: batched time-domain tube synthesis on MI355X.

python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--seconds S] [--fs HZ]
                [--workload static|fricatives|vcv]
For N > 1 either run `python bench.py --gpus N` (it starts the N ranks itself: a child
torch.distributed.run, one rank per GPU) or launch it under torch.distributed.run with --gpus
equal to WORLD_SIZE (anything else is refused).

One *step* = one pass of the hot path over this rank's shard of the metric's batch (BASELINE
config 4: 65536 static-vowel utterances of S seconds at fs Hz, split over the N GPUs -- strong
scaling: 65536 on one GPU, 8192 per GPU at 8; --batch B instead fixes B per GPU, weak scaling),
from frames already resident in HBM to fp64 audio in HBM, converted on the GPU to the reference's
int16 output format and (N > 1) gathered to rank 0 by the library's RCCL gather (afs_gather_pcm,
xGMI) while the next step synthesizes.  torch.distributed (gloo) only carries the control plane:
the RCCL id, barriers and the max-over-ranks time.

Printed (rank 0): one JSON line with the BASELINE metric (whole-node samples/s), the roofline
object of the dominant kernel (HBM, as the north star asks, with the kernel's own launch times
from HIP events around every launch: afs_kernel_times), the fp64 object (the path's binding
resource: algorithmic flops counted from the restatement, profiles/flops_per_sample.json) and
the CPU baseline (the reference's own sources, oracle/_ref, timed on this host's cores over a
bounded sample, plus the single-core config-1 figure).  On one GPU the line also carries
"configs": config 2 (1024 static vowels: one utterance per SIMD, the voice kernel's per-sample
latency), config 5 (8192 fricatives, velum 1.0 cm^2) and config 3 (8192 VCV utterances through
playTargetSequence), each timed over a few steps with its own launch times, roofline, fp64
object, reference CPU rate and error against the reference build, and "config4_shard": config 4's
per-GPU shard at 8 GPUs (8192 utterances; the headline of rounds 1-4), its rows checked bit for
bit against the batch's first rows (--no-sub-configs skips them).
PMC-derived figures are quoted only when profiles/pmc_*.json hold a pass of this build's kernel
sources (areafunctionsynthesis_amd.build.kernel_digest).
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
CPU_PROC_CAP = 16              # the box's CPU share per GPU (gpurun: 16 for one GPU)


def flops_per_sample(workload: str):
    """fp64 flops per sample (tools/flopcount: the restatement in the reference's operation
    order, instrumented; with the own-algorithm figure beside it), for the workload's family."""
    path = os.path.join(ROOT, "profiles", "flops_per_sample.json")
    if not os.path.exists(path):
        return None, None
    db = json.load(open(path))["workloads"]
    fam = {"static": "config2", "fricatives": "config5", "vcv": "config3"}[workload]
    for name, e in db.items():
        if name.startswith(fam):
            return e["per_sample"], name
    return None, None


def pmc_entry(name: str, key: str, digest: str):
    """(entry, stale) of a committed PMC summary under profiles/: the entry measured on this
    build's kernel sources (build.kernel_digest), else (None, the newest other entry's tag)."""
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None, None
    by = json.load(open(path)).get(key) or {}
    if "tag" in by:  # (a summary written before the entries were keyed by the sources' digest)
        by = {"?": by}
    if digest in by:
        return by[digest], None
    others = sorted(by.values(), key=lambda e: e.get("tag", ""))
    return None, (others[-1].get("tag") if others else None)


def frame_bytes_per_sample(hop: int) -> float:
    # one 1072-B frame per hop samples + one 8-B fp64 output sample
    return 1072.0 / hop + 8.0


def _cpu_init():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib  # noqa: F401  (load the libraries before the clock starts)


def _cpu_job(job):
    """One utterance on one core; returns (samples, seconds of compute, audio)."""
    kind, what, data, seed, hop, fs = job
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import Oracle, RefLib
    lib = RefLib() if kind == "reference" else Oracle()
    if what == "target":  # playTargetSequence: per-sample area function -> tube, then n = 1 calls
        t0 = time.perf_counter()
        x = lib.utterance(Oracle().target_frames(data, fs), 1, seed, fs)
    else:
        t0 = time.perf_counter()
        x = lib.utterance(data, hop, seed, fs)
    return x.size, time.perf_counter() - t0, x


def cpu_baseline(jobs, fs: float, n_utt: int, gpu_out: np.ndarray, what: str, config1_frames):
    """The reference build (oracle/_ref; the restatement if it is absent) on a bounded sample of
    the same workload, one process per core, plus config 1 (the `a:` utterance, 1 s, one core).
    The pool is started and warmed before the clock; each job also times its own compute."""
    import multiprocessing as mp

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import REF_SO

    kind = "reference" if os.path.exists(REF_SO) else "port"
    host_cpus = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cores = max(1, min(CPU_PROC_CAP, host_cpus, n_utt))
    jobs = [(kind,) + tuple(j) + (fs,) for j in jobs]
    ctx = mp.get_context("spawn")
    with ctx.Pool(cores, initializer=_cpu_init) as pool:
        pool.map(_cpu_init_probe, range(cores))  # every worker up and its libraries loaded
        t0 = time.perf_counter()
        outs = pool.map(_cpu_job, jobs, chunksize=1)
        wall = time.perf_counter() - t0
        c1 = pool.apply(_cpu_job, ((kind, "frames", config1_frames, 1, 441, fs),))
    samples = sum(o[0] for o in outs)
    busy = sum(o[1] for o in outs)
    errs = [float(np.abs(gpu_out[u] - outs[u][2]).max()) for u in range(n_utt)]
    rmss = [float(np.sqrt(np.mean((gpu_out[u] - outs[u][2]) ** 2))) for u in range(n_utt)]
    per_core = samples / busy
    return {
        "value": samples / wall,
        "unit": "samples/s",
        "cores": cores,
        "kind": kind,
        "sample": f"{n_utt} utterances ({what}) @ {fs:g} Hz (the first utterances of this shard), "
                  f"{cores} worker processes (pool warmed before the clock)",
        "per_core_samples_per_s": per_core,
        "host_cpus": host_cpus,
        "process_cap": CPU_PROC_CAP,
        "whole_host_estimate_samples_per_s": per_core * host_cpus,
        "config1_single_core_samples_per_s": c1[0] / c1[1],
        "config1": f"a: (Default.params), f0 120 Hz, 8000 dPa, 1 s @ {fs:g} Hz, one core, "
                   "Synthesizer.cpp:515-639 driver restated in oracle/ref_harness.cpp",
    }, max(errs), max(rmss)


def _cpu_init_probe(_):
    return os.getpid()


def config1_frames(fs: float):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import Oracle
    from areafunctionsynthesis_amd.frames import DEFAULT_GLOTTIS
    from areafunctionsynthesis_amd.params import default_shapes
    f = Oracle().af_to_frame(default_shapes()["a:"])
    f["glottis"] = DEFAULT_GLOTTIS
    f["glottis"][1] = 8000.0  # sensorDataToGlottisParams (Synthesizer.cpp:905)
    return np.repeat(f[None], int(round(fs / 441)) + 1)


WORKLOAD_TEXT = {
    "static": "BASELINE config 4: {G} static-vowel utterances x {sec:g} s @ {fs:g} Hz over {N} GPU(s), {B} per GPU, "
              "frames resident in HBM",
    "config2": "BASELINE config 2: {B} static-vowel utterances x {sec:g} s @ {fs:g} Hz on one GPU (one utterance per "
               "SIMD: the voice kernel's per-sample latency), frames resident in HBM",
    "fricatives": "BASELINE config 5: {B} fricative utterances (s f z S Z x C R v) + velum 1.0 cm^2 per GPU x "
                  "{sec:g} s @ {fs:g} Hz, frames resident in HBM",
    "vcv": "BASELINE config 3 (fp64 state): {B} VCV utterances/GPU through playTargetSequence ({T} samples @ "
           "{fs:g} Hz, per-sample area-function tubes built on the GPU)",
}


class Measured:
    """One workload's timed run: K steps bracketed by synchronisations (and barriers)."""


def measure(args, ctx, dev, stream, workload: str, B: int, first: int, world: int, rank: int, comm,
            steps: int, warmup: int) -> Measured:
    import torch
    import torch.distributed as dist

    from areafunctionsynthesis_amd import sharding
    from areafunctionsynthesis_amd.frames import FRAME_DTYPE
    from areafunctionsynthesis_amd.workloads import build_frames, fricatives, static_vowels, vcv_targets

    m = Measured()
    m.workload, m.B, m.steps, m.warmup = workload, B, steps, warmup
    m.kernel = ctx.synthesis_kernel(B)  # (the profiler's name of the synthesis kernel this batch runs)
    if workload in ("static", "fricatives"):
        gen = static_vowels if workload == "static" else fricatives
        w = gen(B, seconds=args.seconds, fs=args.fs, first_utterance=first)
        m.frames = build_frames(w, ctx.af_to_frames)
        m.F, m.hop, m.T = w.num_frames, w.hop, w.samples_per_utterance
        m.seeds = w.seeds
        frames_dev = torch.from_numpy(m.frames.view(np.uint8).reshape(B, m.F, FRAME_DTYPE.itemsize)).to(dev)

        def synth():
            ctx.synthesize(frames_dev, m.hop, seeds=seeds_dev, out=out_dev)
    else:
        m.shapes, m.targets, m.seeds = vcv_targets(B, first_utterance=first)
        m.hop, m.T = 1, ctx.target_sequence_samples()
        m.distinct = int(np.unique(m.targets, axis=0).shape[0])  # (one tube trajectory per distinct sequence)

        def synth():
            ctx.play_target_sequences(m.shapes, m.targets, seeds=seeds_dev, out=out_dev)
    seeds_dev = torch.from_numpy(m.seeds.astype(np.int32)).to(dev)
    out_dev = torch.empty((B, m.T), dtype=torch.float64, device=dev)
    m.out_dev = out_dev

    # the reference's output format (int16, Synthesizer.cpp:955-973) is produced on the GPU and
    # gathered to rank 0 by the library's RCCL gather while the next step synthesizes
    if comm is not None:
        transport = sharding.CommTransport(comm)
    elif world > 1:  # (--gather-transport gloo: the test transport, tests/test_multi_gpu.py)
        transport = sharding.StagedTorchTransport(dist, world, rank)
    else:
        transport = _NoGather()
    pcm = sharding.PcmGather(lambda x, o: ctx.to_int16(x, out=o), (B, m.T), world, rank, transport, device=dev)

    for _ in range(warmup):
        synth()
        pcm.submit(out_dev)
    pcm.drain()
    torch.cuda.synchronize(dev)
    ctx.kernel_times()  # drop the warm-up launches
    if comm is not None:
        comm.gather_times()  # (and the warm-up gathers)

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(steps):
        ev[k][0].record(stream)
        synth()
        ev[k][1].record(stream)
        pcm.submit(out_dev)
        ev[k][2].record(stream)
    pcm.drain()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    m.synth_ms = [a.elapsed_time(b) for a, b, _ in ev]
    m.int16_ms = [b.elapsed_time(c) for _, b, c in ev]  # (the int16 conversion, and at N > 1 its gather's enqueue)
    m.kt = ctx.kernel_times()
    t = torch.tensor([elapsed], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    m.elapsed = float(t.item())
    m.multi = None
    if world > 1:
        # the slowest rank's kernel and gather times (HIP events; the gathers on the comm's stream)
        gt = comm.gather_times() if comm is not None else {"gather_ms": 0.0, "gathers": 0}
        launches = max(1, m.kt["synth_launches"])
        mx = torch.tensor([m.kt["synth_ms"] / launches, gt["gather_ms"] / steps], dtype=torch.float64)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        m.multi = {"avg_launch_ms_max_over_ranks": float(mx[0]), "gather_ms_per_step_max_over_ranks": float(mx[1]),
                   "gathers_per_step_rank0": gt["gathers"] / steps,
                   "transport": "rccl (afs_gather_pcm)" if comm is not None else "gloo via the host (test transport)",
                   "gather_timing": "HIP events on the comm's stream around each afs_gather_pcm "
                                    "(afs_comm_gather_times); the gather overlaps the next step's synthesis"}
        # self-check of the exchange: rank 0 compares the int16 rows it received (the last step's
        # slot) with the same utterances synthesized on rank 0 alone
        if rank == 0:
            edges = sharding.edge_utterances(world, B)
            root = pcm.result((pcm.k - 1) % len(pcm.bufs))
            rows = torch.stack([root[r, j] for r, j, _ in edges]).cpu()
            # (the re-synthesis uses the kernel the shards ran: the lane width chosen for B, not for
            # the few utterances re-synthesized)
            from areafunctionsynthesis_amd.synthesizer import Context
            lanes = ctx.lanes_per_utterance(B) if args.solver == "tree" else None
            chk = Context(args.fs, solver=args.solver, device=ctx.device, lanes=lanes)
            try:
                m.gather_check = sharding.check_gathered(rows, world, B, lambda us: _resynth(chk, m, us, args))
            finally:
                chk.close()
            m.gather_check["lanes_per_utterance"] = lanes
        dist.barrier()
    return m


def _resynth(ctx, m, us, args):
    """int16 audio [len(us), T] of global utterances `us` synthesized on this GPU in one call
    (the frames / targets and seeds u + 1 the full batch gives them)."""
    from areafunctionsynthesis_amd.workloads import build_frames, fricatives, static_vowels, vcv_targets
    seeds = np.array([u + 1 for u in us], dtype=np.uint32)
    if m.workload in ("static", "fricatives"):
        gen = static_vowels if m.workload == "static" else fricatives
        frames = np.concatenate([build_frames(gen(1, seconds=args.seconds, fs=args.fs, first_utterance=u),
                                              ctx.af_to_frames) for u in us])
        y = ctx.synthesize(frames, m.hop, seeds=seeds)
    else:
        shapes, _, _ = vcv_targets(1)
        targets = np.concatenate([vcv_targets(1, first_utterance=u)[1] for u in us])
        y = ctx.play_target_sequences(shapes, targets, seeds=seeds)
    return ctx.to_int16(y)


def describe(args, m: Measured, world: int, digest: str) -> dict:
    """value, roofline and fp64 objects of a measured workload."""
    B, T, hop = m.B, m.T, m.hop
    total_samples = float(world) * B * T * m.steps
    value = total_samples / m.elapsed
    kname = m.kernel
    launches = max(1, m.kt["synth_launches"])
    avg_launch_s = m.kt["synth_ms"] / launches / 1e3
    samples_per_launch = B * T * m.steps / launches
    bps = frame_bytes_per_sample(hop)
    alg_bytes = samples_per_launch * bps
    achieved_gbs = alg_bytes / avg_launch_s / 1e9
    tkey = f"{kname}|{m.workload}|B={B}|T={T}|hop={hop}"
    tr, tr_stale = pmc_entry("pmc_traffic.json", tkey, digest)
    sq, sq_stale = pmc_entry("pmc_sq_fp64.json", tkey, digest)
    per, per_src = flops_per_sample(m.workload)
    fp64 = None
    if per is not None:
        alg_tf = per["flops"] * samples_per_launch / avg_launch_s / 1e12
        own = per.get("own_algorithm_flops")
        own_tf = own * samples_per_launch / avg_launch_s / 1e12 if own else None
        fp64 = {
            "algorithmic_flops_per_sample": per["flops"],
            "algorithmic_transcendentals_per_sample": per["transc"],
            "algorithmic_source": f"profiles/flops_per_sample.json [{per_src}]: the restatement in the "
                                  "reference's operation order (envelope Cholesky), instrumented per IR block",
            "achieved_tflops": alg_tf,
            "peak_tflops": FP64_PEAK_TFLOPS,
            "frac": alg_tf / FP64_PEAK_TFLOPS,
            "own_algorithm_flops_per_sample": own,
            "own_algorithm": "the same count with the envelope Cholesky (counted per function: "
                             f"{per.get('cholesky_flops', 0):.0f} flops) replaced by the arm LDL^T "
                             f"({per.get('arm_ldlt_flops', 0):.0f} flops: 2 per current, 7 per edge)",
            "own_algorithm_achieved_tflops": own_tf,
            "own_algorithm_frac": own_tf / FP64_PEAK_TFLOPS if own_tf else None,
            "executed_lane_flops_per_sample": sq["lane_flops_per_sample"] if sq else None,
            "executed_source": (f"profiles/pmc_sq_fp64.json [{sq['tag']}, commit {sq.get('commit')}, sources "
                                f"{digest} = this build] (SQ_INSTS_VALU_FLOPS_FP64 x 64 lanes / 4 utterances per wave)"
                                if sq else (f"no SQ pass of this build's kernel (sources {digest}); newest is "
                                            f"{sq_stale}" if sq_stale else None)),
        }
    roof = {
        "bound": "hbm",
        "achieved": achieved_gbs,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": achieved_gbs / HBM_PEAK_GBS,
        "traffic": tr["traffic_bytes_per_launch"] if tr else None,
        "traffic_unit": "bytes per launch (rocprofv3 PMC)",
        "traffic_correction": tr["correction"] if tr else None,
        "traffic_source": (f"profiles/pmc_traffic.json [{tr['tag']}, commit {tr.get('commit')}, sources {digest} = "
                           "this build]" if tr else (f"no PMC pass of this build's kernel (sources {digest}); "
                                                     f"newest is {tr_stale}" if tr_stale else None)),
        "algorithmic_bytes_per_launch": alg_bytes,
        "bytes_per_sample": bps,
        "kernel": kname,
        "avg_launch_ms": avg_launch_s * 1e3,
        "launches_per_step": m.kt["synth_launches"] / m.steps,
        "launch_timing": "HIP events around every launch on the library's stream (afs_kernel_times)",
        "plan_kernel_ms_per_step": m.kt["plan_ms"] / m.steps,
        "output_kernel_ms_per_launch": m.kt["output_ms"] / max(1, m.kt["output_launches"]),
        "output_kernel": "tree_output_kernel (K6: glottal-tone filter + dU/dt + Chebyshev low-pass after each K1 launch)",
        "binding_resource": "neither HBM nor MFMA: the latency of the per-sample fp64 recurrence "
                            "(SURVEY.md 8(d)); see fp64",
    }
    if m.workload == "vcv":
        # hop 1: every utterance reads its trajectory's frame each sample, but the batch plays only
        # `distinct` trajectories (afs_play_target_sequences builds one per distinct target sequence)
        roof["algorithmic_bytes_meaning"] = (
            "per-utterance bytes: one 1072-B frame per utterance-sample (hop 1) + the 8-B output sample; "
            f"the {B} utterances play {m.distinct} distinct trajectories, so the distinct frame bytes are "
            "far fewer (distinct_frame_bytes_per_launch) and most frame reads hit the caches -- the "
            "achieved GB/s above is a per-utterance rate, not HBM traffic (that is `traffic`)")
        roof["distinct_trajectories"] = m.distinct
        roof["distinct_frame_bytes_per_launch"] = float(m.distinct) * samples_per_launch / B * 1072.0
    if tr and tr.get("plan_kernel_traffic_bytes_per_launch") is not None:
        roof["plan_kernel_traffic_bytes_per_launch"] = tr["plan_kernel_traffic_bytes_per_launch"]
    ms_step = m.elapsed / m.steps * 1e3
    dev_ms, i16_ms = float(np.mean(m.synth_ms)), float(np.mean(m.int16_ms))
    return {"value": value, "ms_per_step": ms_step, "roofline": roof, "fp64": fp64,
            "step_device_ms": dev_ms, "int16_ms_per_step": i16_ms, "idle_ms_per_step": ms_step - dev_ms - i16_ms,
            "sq": sq}


def cpu_leg(args, m: Measured, n: int):
    """The reference build on the first n utterances of the measured batch (bounded sample)."""
    gpu_out = m.out_dev[:n].cpu().numpy()
    if m.workload != "vcv":
        jobs = [("frames", m.frames[u], int(m.seeds[u]), m.hop) for u in range(n)]
        what = f"{m.F - 1} frames x {m.hop} samples"
    else:
        jobs = [("target", m.shapes[m.targets[u]], int(m.seeds[u]), None) for u in range(n)]
        what = f"playTargetSequence, {m.T} samples, trajectory built per sample on the CPU"
    return cpu_baseline(jobs, args.fs, n, gpu_out, what, config1_frames(args.fs))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of this node; default: WORLD_SIZE, else 1.  Without WORLD_SIZE, "
                         "--gpus N > 1 starts the N ranks itself (torch.distributed.run as a child process)")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--global-batch", type=int, default=65536,
                    help="the metric's batch (BASELINE config 4: 65536 utterances), split over the GPUs (strong "
                         "scaling: 65536 on one GPU, 8192 per GPU at 8)")
    ap.add_argument("--batch", type=int, default=None,
                    help="utterances per GPU instead (weak scaling; the global batch is then batch x GPUs)")
    ap.add_argument("--sub-batch", type=int, default=8192,
                    help="one GPU: utterances of the config-5 / config-3 sub-objects (BASELINE: 8192) and of the "
                         "config-4 per-GPU shard sub-object")
    ap.add_argument("--seconds", type=float, default=1.0)
    ap.add_argument("--fs", type=float, default=44100.0)
    ap.add_argument("--solver", default=os.environ.get("AFS_SOLVER", "tree"))
    ap.add_argument("--cpu-utterances", type=int, default=128,
                    help="CPU baseline: utterances of the headline's bounded sample (128 x 1 s: ~38 core-seconds of "
                         "the reference's work, ~2.5 s on the box's 16-CPU share)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", choices=("static", "fricatives", "vcv"), default="static",
                    help="static: config-4 shard of static vowels (default); fricatives: config 5 "
                         "(fricatives + velum 1.0 cm^2); vcv: config-3 VCV utterances through "
                         "playTargetSequence (per-sample tubes, hop 1)")
    ap.add_argument("--no-sub-configs", action="store_true",
                    help="skip the config-5 / config-3 sub-objects (one GPU, default workload only)")
    ap.add_argument("--lanes", type=int, choices=(16, 64), default=None,
                    help="tree solver: force 16 (throughput kernel) or 64 (voice kernel) lanes per utterance; "
                         "default: the library's choice for the batch")
    ap.add_argument("--sub-steps", type=int, default=2)
    ap.add_argument("--config2-batch", type=int, default=1024,
                    help="one GPU: utterances of the config-2 sub-object (BASELINE config 2: 1024 static vowels)")
    ap.add_argument("--gather-transport", choices=("rccl", "gloo"), default="rccl",
                    help="N > 1: rccl (the library's afs_gather_pcm; default) or gloo through the host (test only)")
    ap.add_argument("--one-device", action="store_true",
                    help="N > 1: every rank on device 0 (test of the multi-process path on a one-GPU box)")
    ap.add_argument("--sub-cpu-utterances", type=int, default=48)
    ap.add_argument("--pg-timeout", type=float, default=300.0,
                    help="N > 1: seconds a rank waits in a control-plane collective before failing")
    ap.add_argument("--launch-check", action="store_true",
                    help="N > 1 test option: start the ranks and the process group, print the world, no GPU work")
    ap.add_argument("--fail-rank", type=int, default=None,
                    help="N > 1 test option: this rank raises after the process group is up")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        # `python bench.py --gpus N`: start the N ranks ourselves, as a child torch.distributed.run,
        # before this process makes any GPU call (none follows either)
        sys.exit(_launch_ranks(args.gpus))
    world = int(env_world or "1")
    if args.gpus is not None and args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import datetime

    import torch
    import torch.distributed as dist

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=args.pg_timeout))
        if args.fail_rank == rank:
            raise RuntimeError(f"bench.py: rank {rank} fails on request (--fail-rank)")
        if args.launch_check:
            t = torch.ones(1)
            dist.all_reduce(t)
            if rank == 0:
                print(json.dumps({"launch_check": True, "n_gpus": world, "ranks_reporting": int(t.item())}),
                      flush=True)
            dist.barrier()
            dist.destroy_process_group()
            return
    if args.one_device:
        local = 0
    elif torch.cuda.device_count() < world:  # (counting devices initialises no GPU)
        print(f"bench.py: {world} ranks but {torch.cuda.device_count()} visible GPUs", file=sys.stderr)
        sys.exit(3)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from areafunctionsynthesis_amd import sharding
    from areafunctionsynthesis_amd.build import kernel_digest
    from areafunctionsynthesis_amd.synthesizer import Comm, Context, comm_unique_id

    digest = kernel_digest()
    if args.batch is None and args.workload != "static":  # (configs 5 and 3: 8192 utterances per GPU)
        args.batch = args.sub_batch
    if args.batch is None:  # strong scaling: the metric's batch over the GPUs
        if args.global_batch % world:
            print(f"bench.py: --global-batch {args.global_batch} does not split over {world} GPUs", file=sys.stderr)
            sys.exit(2)
        B, scaling = args.global_batch // world, "strong"
    else:
        B, scaling = args.batch, "weak"
    ctx = Context(args.fs, solver=args.solver, device=local, async_calls=True, profile=True, lanes=args.lanes)
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)
    first, _ = sharding.shard_range(rank, world, B)
    comm = None
    if world > 1 and args.gather_transport == "rccl":
        uid = [comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = Comm(ctx, uid[0], rank, world)

    m = measure(args, ctx, dev, stream, args.workload, B, first, world, rank, comm, args.steps, args.warmup)
    # one GPU: config 5 and config 3 are timed too (sub-objects, a few steps each)
    subs = []
    if world == 1 and args.workload == "static" and not args.no_sub_configs:
        # config 2 (1024 static vowels: one utterance per SIMD, the voice kernel's per-sample latency)
        subs.append(("config2", measure(args, ctx, dev, stream, "static", args.config2_batch, 0, world, rank, None,
                                        args.sub_steps, 1)))
        for wl, label in (("fricatives", "config5"), ("vcv", "config3")):
            subs.append((label, measure(args, ctx, dev, stream, wl, args.sub_batch, 0, world, rank, None,
                                        args.sub_steps, 1)))
    # one GPU: config 4's per-GPU shard at 8 GPUs (8192 utterances), the headline of rounds 1-4
    shard = None
    if world == 1 and args.workload == "static" and not args.no_sub_configs and args.sub_batch != B:
        shard = measure(args, ctx, dev, stream, "static", args.sub_batch, 0, 1, 0, None, args.sub_steps, 1)
        n = min(B, args.sub_batch)
        # batch independence: the shard's utterances are the batch's first ones, bit for bit
        shard.same_as_batch = bool(torch.equal(shard.out_dev[:n], m.out_dev[:n]))
        shard.same_rows = n

    if rank == 0:
        d = describe(args, m, world, digest)
        result = {
            "metric": "audio samples/s (whole node) on 64k-utterance batch; max-abs err vs CPU ref",
            "value": d["value"],
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": d["ms_per_step"],
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": WORKLOAD_TEXT[args.workload].format(B=B, G=B * world, N=world, sec=args.seconds,
                                                                fs=args.fs, T=m.T),
                "batch_per_gpu": B,
                "global_batch": B * world,
                "samples_per_utterance": m.T,
                "fs_hz": args.fs,
                "hop": m.hop,
                "solver": args.solver,
                "lanes_per_utterance": ctx.lanes_per_utterance(B),
                "kernel_sources": digest,
                "parallelism": f"dp{world} (utterance shards; int16 audio gathered to rank 0 by afs_gather_pcm over "
                               "RCCL, overlapped with the next step)" if world > 1 else "dp1",
            },
            "x_realtime": d["value"] / args.fs,
            "step_device_ms": d["step_device_ms"],
            "int16_ms_per_step": d["int16_ms_per_step"],
            # (the step's wall time not covered by its device work: host waits and launch gaps; HIP events on
            # the library's stream around the synthesis call and the int16 conversion)
            "idle_ms_per_step": d["idle_ms_per_step"],
            "roofline": d["roofline"],
            "fp64": d["fp64"],
        }
        if world > 1:
            result["multi_gpu"] = m.multi
            result["gather_check"] = m.gather_check
        if world > 1 and not args.no_cpu_baseline:
            # (no CPU timing at N > 1: the error of rank 0's first utterances against the reference build)
            _, max_abs, max_rms = cpu_leg(args, m, min(8, B))
            result["max_abs_err_vs_cpu_ref"] = max_abs
            result["max_rms_err_vs_cpu_ref"] = max_rms
            result["cpu_ref_utterances"] = min(8, B)
        if world == 1 and not args.no_cpu_baseline:
            cb, max_abs, max_rms = cpu_leg(args, m, min(args.cpu_utterances, B))
            result["cpu_baseline"] = cb
            result["max_abs_err_vs_cpu_ref"] = max_abs
            result["max_rms_err_vs_cpu_ref"] = max_rms
        if subs:
            result["configs"] = {}
            for label, ms in subs:
                ds = describe(args, ms, world, digest)
                text = WORKLOAD_TEXT["config2" if label == "config2" else ms.workload]
                o = {
                    "workload": text.format(B=ms.B, G=ms.B, N=1, sec=args.seconds, fs=args.fs, T=ms.T),
                    "batch": ms.B,
                    "value": ds["value"], "unit": "samples/s", "steps": ms.steps, "warmup": ms.warmup,
                    "ms_per_step": ds["ms_per_step"], "samples_per_utterance": ms.T, "hop": ms.hop,
                    "lanes_per_utterance": ctx.lanes_per_utterance(ms.B),
                    "avg_launch_ms": ds["roofline"]["avg_launch_ms"], "roofline": ds["roofline"], "fp64": ds["fp64"],
                }
                if ds.get("sq"):
                    o["cycles_per_wave_sample"] = ds["sq"]["wave_cycles_per_wave_sample"]
                    o["utterances_per_wave"] = ds["sq"].get("utterances_per_wave", 4)
                    o["cycles_source"] = ds["fp64"]["executed_source"] if ds["fp64"] else None
                if label == "config2":
                    # the voice kernel's per-sample latency: one utterance per wave, one wave per SIMD
                    o["us_per_sample_per_utterance"] = ds["roofline"]["avg_launch_ms"] * 1e3 / (
                        ms.T / max(1.0, ds["roofline"]["launches_per_step"]))
                if not args.no_cpu_baseline:
                    cb, max_abs, max_rms = cpu_leg(args, ms, min(args.sub_cpu_utterances, ms.B))
                    o["cpu_reference_per_core_samples_per_s"] = cb["per_core_samples_per_s"]
                    o["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind", "sample",
                                                            "per_core_samples_per_s")}
                    o["max_abs_err_vs_cpu_ref"] = max_abs
                    o["max_rms_err_vs_cpu_ref"] = max_rms
                result["configs"][label] = o
        if shard is not None:
            ds = describe(args, shard, 1, digest)
            result.setdefault("configs", {})["config4_shard"] = {
                "workload": f"BASELINE config 4's per-GPU shard at 8 GPUs: {shard.B} static-vowel utterances x "
                            f"{args.seconds:g} s @ {args.fs:g} Hz on this GPU (the headline of rounds 1-4)",
                "batch": shard.B, "value": ds["value"], "unit": "samples/s", "steps": shard.steps,
                "warmup": shard.warmup, "ms_per_step": ds["ms_per_step"],
                "avg_launch_ms": ds["roofline"]["avg_launch_ms"],
                "launches_per_step": ds["roofline"]["launches_per_step"],
                "ratio_to_value": ds["value"] / d["value"],
                "roofline": ds["roofline"], "fp64": ds["fp64"],
                "rows_bitwise_equal_to_the_batch": shard.same_as_batch, "rows_compared": shard.same_rows,
                "why_slower": "8192 utterances are two rounds of workgroups per CU slot (65536: sixteen); K1 takes "
                              "~159 ms per round of 0.5 s utterances plus a fixed ~21-29 ms per launch, present with "
                              "uniform blocks too -- 8 % of an 8192 launch, 1 % of a 65536 one (DESIGN.md 2.5)",
            }
        print(json.dumps(result), flush=True)
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


def _launch_ranks(n: int) -> int:
    """Run this command as N ranks: `python -m torch.distributed.run --nproc-per-node N bench.py
    <the same arguments>` in a child process (never an exec: this process stays GPU-free), rank 0's
    JSON line reaching our stdout through the inherited descriptor.  torch.distributed.run ends
    every rank when one fails, so a failing rank makes the whole command exit non-zero; the
    return code is the child's."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, env=env)
    return r.returncode


class _NoGather:
    """One GPU: the int16 audio is already whole on rank 0."""

    def gather(self, slot, local, root):
        pass

    def fence(self, slot):
        pass

    def drain(self):
        pass


if __name__ == "__main__":
    main()
