"""Large tree calls without host read-backs (afs_capi.cpp shape_order, run_chunks): the slot order is
sorted on the device, and K5's compact mixed-hop slots are sized up front, the synthesis launches
guarded on the device by the count K5 claimed.  Two AFS_ASYNC calls of 8192 utterances are queued
back to back on one stream:

  * with the worst case of mixed hops inside the plan budget (AFS_PLAN_BUDGET_MB raised), neither
    call waits for the device: both return while the first call's synthesis kernel still runs;
  * with the default budget (the worst case past it), a call waits for its own K5 after its launches
    are queued -- the device never idles between the calls: the first call returns before its
    synthesis ends, and the time between the two calls' work on the device is below 1 ms;
  * the audio is the same bit for bit as one synchronous call of each batch, and the guarded
    fallback (K5's slots overflowing a small budget) gives the same audio too.
"""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

B = 8192
SECONDS = 0.25


def _setup(ctx, first):
    import torch

    from areafunctionsynthesis_amd.frames import FRAME_DTYPE
    from areafunctionsynthesis_amd.workloads import build_frames, static_vowels
    w = static_vowels(B, seconds=SECONDS, fs=44100.0, first_utterance=first)
    frames = build_frames(w, ctx.af_to_frames)
    dev = torch.device("cuda", 0)
    f = torch.from_numpy(frames.view(np.uint8).reshape(B, w.num_frames, FRAME_DTYPE.itemsize)).to(dev)
    s = torch.from_numpy(w.seeds.astype(np.int32)).to(dev)
    o = torch.empty((B, w.samples_per_utterance), dtype=torch.float64, device=dev)
    return w, f, s, o


def _two_calls(monkeypatch, budget_mb):
    import torch

    from areafunctionsynthesis_amd.synthesizer import Context
    if budget_mb:
        monkeypatch.setenv("AFS_PLAN_BUDGET_MB", str(budget_mb))
    else:
        monkeypatch.delenv("AFS_PLAN_BUDGET_MB", raising=False)
    ctx = Context(44100.0, solver="tree", async_calls=True, profile=True)
    try:
        stream = torch.cuda.current_stream()
        ctx.set_stream(stream.cuda_stream)
        (w1, f1, s1, o1), (w2, f2, s2, o2) = _setup(ctx, 0), _setup(ctx, B)
        torch.cuda.synchronize()
        # one call alone (after a warm-up): its device span, every kernel of the call included
        ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(2):
            ea.record(stream)
            ctx.synthesize(f2, w2.hop, seeds=s2, out=o2)
            eb.record(stream)
            torch.cuda.synchronize()
        one = ea.elapsed_time(eb)
        ctx.kernel_times()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e2 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        t0 = time.perf_counter()
        ctx.synthesize(f1, w1.hop, seeds=s1, out=o1)
        e1.record(stream)
        t1 = time.perf_counter()
        first_running_after_call1 = not e1.query()
        ctx.synthesize(f1, w1.hop, seeds=s1, out=o2)  # (the same batch again: the same device work)
        t2 = time.perf_counter()
        first_running_after_call2 = not e1.query()
        e2.record(stream)
        second_running_after_call2 = not e2.query()
        torch.cuda.synchronize()
        kt = ctx.kernel_times()
        span = e0.elapsed_time(e2)
        busy = kt["synth_ms"] + kt["plan_ms"] + kt["output_ms"]
        res = {"call1_ms": (t1 - t0) * 1e3, "call2_ms": (t2 - t1) * 1e3, "span_ms": span, "busy_ms": busy,
               "one_call_span_ms": one, "gap_ms": span - 2 * one,
               "first_running_after_call1": first_running_after_call1,
               "first_running_after_call2": first_running_after_call2,
               "second_running_after_call2": second_running_after_call2, "k1_ms": kt["synth_ms"]}
        # the same audio as a synchronous call of each batch on a fresh context
        ref = Context(44100.0, solver="tree")
        try:
            y1 = ref.synthesize(f1, w1.hop, seeds=s1, out=torch.empty_like(o1))
            torch.cuda.synchronize()
            res["same"] = bool(torch.equal(y1, o1)) and bool(torch.equal(y1, o2))
        finally:
            ref.close()
        return res
    finally:
        ctx.close()


def test_two_async_calls_no_host_wait(monkeypatch, parity_report):
    # worst case of mixed hops: 8192 x 25 hops x 441 x 128 B = 11.6 GB of slots
    r = _two_calls(monkeypatch, 16384)
    parity_report.append(
        f"two AFS_ASYNC calls of {B} static vowels x {SECONDS:g} s, mixed-hop slots for the worst case (budget 16 GB): "
        f"call 1 returned in {r['call1_ms']:.2f} ms, call 2 in {r['call2_ms']:.2f} ms while the first call's "
        f"synthesis ({r['k1_ms'] / 2:.0f} ms per call) still ran: {r['first_running_after_call2']}; device span "
        f"{r['span_ms']:.2f} ms vs 2 x {r['one_call_span_ms']:.2f} ms of one call alone (idle {r['gap_ms']:.3f} ms); "
        f"audio bitwise as synchronous calls: {r['same']}")
    assert r["first_running_after_call1"] and r["first_running_after_call2"], r
    assert r["same"]


def test_two_async_calls_default_budget(monkeypatch, parity_report):
    r = _two_calls(monkeypatch, 0)
    parity_report.append(
        f"two AFS_ASYNC calls of {B} static vowels x {SECONDS:g} s, default plan budget (each call waits for its own "
        f"K5 after queueing its launches): call 1 returned in {r['call1_ms']:.2f} ms (its synthesis still running: "
        f"{r['first_running_after_call1']}), call 2 in {r['call2_ms']:.2f} ms (its synthesis still running: "
        f"{r['second_running_after_call2']}); device span of the two {r['span_ms']:.2f} ms vs 2 x {r['one_call_span_ms']:.2f} "
        f"ms of one call alone: the device idled {r['gap_ms']:.3f} ms between them; bitwise: {r['same']}")
    assert r["first_running_after_call1"] and r["second_running_after_call2"], r
    assert r["gap_ms"] < 1.0, r
    assert r["same"]


def test_guarded_fallback_on_overflow(monkeypatch):
    """A plan budget that holds the call's hop records but few compact slots (16 MB: 297 slots of 441
    samples): frame-rate VCV trajectories (~7 % of their hops mixed) overflow it, the guarded launches
    do nothing and the call runs through the chunked path -- the same audio as with room for every
    mixed hop (8 GB: no guard)."""
    import torch

    from areafunctionsynthesis_amd.frames import FRAME_DTYPE
    from areafunctionsynthesis_amd.synthesizer import Context
    from areafunctionsynthesis_amd.workloads import build_frames, vcv
    outs, launches = [], []
    for mb in ("16", "8192"):
        monkeypatch.setenv("AFS_PLAN_BUDGET_MB", mb)
        ctx = Context(44100.0, solver="tree", profile=True)
        try:
            w = vcv(256, fs=44100.0)
            frames = build_frames(w, ctx.af_to_frames)
            f = torch.from_numpy(frames.view(np.uint8).reshape(w.batch, w.num_frames, FRAME_DTYPE.itemsize)).cuda()
            y = ctx.synthesize(f, w.hop, seeds=w.seeds,
                               out=torch.empty((w.batch, w.samples_per_utterance), dtype=torch.float64, device="cuda"))
            torch.cuda.synchronize()
            outs.append(y.cpu())
            launches.append(ctx.kernel_times()["synth_launches"])
        finally:
            ctx.close()
    assert launches[1] == 1 and launches[0] > 2, launches  # (the skipped launch, then the chunked path's)
    assert torch.equal(outs[0], outs[1])
