"""The metric's own batch on one GPU (BASELINE.json `metric`): 65 536
static vowels x 1 s @ 44.1 kHz in ONE afs_synthesize call, the call bench.py times.

It exercises what only that size reaches: 16 waves per SIMD, the noise-phase variants chosen by the
call rule at that size, K5's compact mixed-hop slots and the plan budget at 65 536
rows x 100 hops.  Checked:
  * no utterance is flagged non-finite;
  * every 1024th utterance (64) against the oracle over the whole second: per-utterance RMS < 1e-4
    (the north-star bound) and the same rand() call count (a noise source switching at another
    sample would change it, TdsModel.cpp:1647-1666);
  * the first 8192 rows bit for bit equal to a separate 8192-utterance call (the per-GPU shard at 8
    GPUs: batch independence at the sizes the scaling run uses).
Inputs and outputs stay in HBM (torch tensors through the C ABI); only the compared rows cross to the
host.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RMS_TOL = 1e-4
B_METRIC = 65536
B_SHARD = 8192
STRIDE = 1024


def test_metric_batch_65536_one_call(parity_report):
    import torch

    from oracle_lib import oracle_parallel

    from areafunctionsynthesis_amd.frames import FRAME_DTYPE
    from areafunctionsynthesis_amd.synthesizer import Context
    from areafunctionsynthesis_amd.workloads import build_frames, static_vowels

    dev = torch.device("cuda", 0)
    ctx = Context(44100.0, solver="tree", device=0)
    try:
        assert ctx.lanes_per_utterance(B_METRIC) == 16
        w = static_vowels(B_METRIC, seconds=1.0, fs=44100.0)
        frames = build_frames(w, ctx.af_to_frames)
        F, hop, T = w.num_frames, w.hop, w.samples_per_utterance
        fdev = torch.from_numpy(frames.view(np.uint8).reshape(B_METRIC, F, FRAME_DTYPE.itemsize)).to(dev)
        seeds = torch.from_numpy(w.seeds.astype(np.int32)).to(dev)
        out = torch.empty((B_METRIC, T), dtype=torch.float64, device=dev)
        nonfinite = torch.zeros(B_METRIC, dtype=torch.uint8, device=dev)
        _, rep = ctx.synthesize(fdev, hop, seeds=seeds, out=out, report=True, nonfinite=nonfinite)
        torch.cuda.synchronize(dev)
        assert rep["nonfinite_utterances"] == 0
        assert int(nonfinite.sum().item()) == 0
        draws = ctx.rng_draws(B_METRIC)

        idx = np.arange(0, B_METRIC, STRIDE)
        y = out[torch.from_numpy(idx).to(dev)].cpu().numpy()
        x, xd = oracle_parallel(frames[idx], hop, w.seeds[idx], w.fs)
        err = y - x
        rms = np.sqrt(np.mean(err ** 2, axis=1))
        flips = int(np.count_nonzero(draws[idx] != xd))

        # the per-GPU shard at 8 GPUs, synthesized alone: the same rows bit for bit
        shard = torch.empty((B_SHARD, T), dtype=torch.float64, device=dev)
        ctx.synthesize(fdev[:B_SHARD], hop, seeds=seeds[:B_SHARD], out=shard)
        torch.cuda.synchronize(dev)
        same = bool(torch.equal(shard, out[:B_SHARD]))
        parity_report.append(
            f"config 4, the metric's batch in one call [tree16]: {B_METRIC} utterances x {T} samples, "
            f"{rep['device_ms']:.0f} ms on the device ({B_METRIC * T / max(rep['device_ms'], 1e-9) / 1e3:.1f} M samples/s); "
            f"non-finite 0; {len(idx)} utterances (every {STRIDE}th) vs oracle: per-utterance RMS max {rms.max():.2e} "
            f"median {np.median(rms):.2e}, max |err| {np.abs(err).max():.2e}; rand() call counts differing: {flips} "
            f"(oracle total {int(xd.sum())}); first {B_SHARD} rows bitwise equal to a {B_SHARD}-utterance call: {same}")
        for k, u in enumerate(idx):
            assert rms[k] < RMS_TOL, (int(u), float(rms[k]))
        assert flips == 0
        assert same
    finally:
        ctx.close()
