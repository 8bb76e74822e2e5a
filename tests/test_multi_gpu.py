"""Several GPUs through the C ABI (afs_comm_*, afs_gather_pcm, afs_multi_synthesize) and the
launch timing bench.py reads (afs_kernel_times).

The GPU box has one device, so the RCCL communicators here have one rank: the gather is the
local copy and afs_multi_synthesize runs one shard.  That still drives every library call of
the multi-GPU path on the hardware (RCCL loaded and initialised, the gather's stream and
events, the shard offsets); the N > 1 exchange itself is covered by the loopback test of the
same gather logic (tests/test_distributed.py) and is unmeasured on hardware.
"""
import numpy as np
import pytest

from areafunctionsynthesis_amd.frames import DEFAULT_GLOTTIS
from areafunctionsynthesis_amd.params import default_shapes

pytestmark = pytest.mark.gpu


def _frames(oracle, B, F):
    sh = default_shapes()
    names = ("a:", "s", "i:", "f", "u:")
    frames = np.stack([np.repeat(oracle.af_to_frame(sh[names[u % len(names)]])[None], F) for u in range(B)])
    frames["glottis"] = DEFAULT_GLOTTIS
    frames["glottis"][:, :, 0] += np.arange(B)[:, None]
    frames["velum_opening_cm2"][1::2] = 0.5
    return frames


def test_kernel_times_count_every_launch(oracle):
    from areafunctionsynthesis_amd.synthesizer import Context
    ctx = Context(44100.0, profile=True)
    frames = _frames(oracle, 6, 5)
    ctx.synthesize(frames, 441)
    kt = ctx.kernel_times()
    assert kt["synth_launches"] >= 1 and kt["synth_ms"] > 0.0
    assert kt["plan_launches"] == kt["synth_launches"]  # one noise-source plan per tree launch
    assert kt["output_launches"] == kt["synth_launches"] and kt["output_ms"] > 0.0  # K6 after every K1
    assert ctx.kernel_times() == {"synth_ms": 0.0, "synth_launches": 0, "plan_ms": 0.0, "plan_launches": 0,
                                  "output_ms": 0.0, "output_launches": 0}
    ctx.close()
    plain = Context(44100.0)
    with pytest.raises(Exception):
        plain.kernel_times()  # AFS_PROFILE off
    plain.close()


def test_comm_gather_one_rank():
    import torch
    from areafunctionsynthesis_amd.synthesizer import Comm, Context, comm_unique_id
    ctx = Context(44100.0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    comm = Comm(ctx, comm_unique_id(), 0, 1)
    x = torch.arange(-5000, 5000, dtype=torch.int16, device="cuda")
    root = torch.zeros_like(x)
    comm.gather_pcm(x, root)
    comm.fence()
    comm.synchronize()
    assert torch.equal(root, x)
    t = comm.gather_times()  # (afs_comm_gather_times: events on the comm's stream)
    assert t["gathers"] == 1 and t["gather_ms"] >= 0.0
    assert comm.gather_times() == {"gather_ms": 0.0, "gathers": 0}
    comm.close()
    ctx.close()


def test_multi_synthesize_equals_single_device(oracle):
    """afs_multi_synthesize (shard, synthesize, int16, RCCL gather) over the box's device gives
    the int16 audio of afs_synthesize + afs_to_int16, with global seeds u + 1."""
    from areafunctionsynthesis_amd.synthesizer import Context, Node
    B, F, hop = 7, 4, 300
    frames = _frames(oracle, B, F)
    node = Node(44100.0, [0])
    pcm, rep = node.synthesize(frames, hop, report=True)
    ctx = Context(44100.0)
    y = ctx.synthesize(frames, hop)
    ref = ctx.to_int16(y)
    assert pcm.shape == (B, (F - 1) * hop)
    assert np.array_equal(pcm, ref)
    assert rep["samples"] == B * (F - 1) * hop and rep["nonfinite_utterances"] == 0
    seeds = np.arange(11, 11 + B, dtype=np.uint32)
    assert np.array_equal(node.synthesize(frames, hop, seeds=seeds), ctx.to_int16(ctx.synthesize(frames, hop, seeds=seeds)))
    node.close()
    ctx.close()


def test_multi_synthesize_lane_width_of_the_whole_batch(oracle):
    """afs_multi_synthesize runs every shard at the lane width chosen for the whole batch (the two
    widths agree within the tolerances, not bit for bit, so a per-shard choice would make the audio
    depend on the GPU count): a batch above the SIMD count gives the 16-lane kernel's audio, one
    below it the 64-lane kernel's, bit for bit."""
    from areafunctionsynthesis_amd.synthesizer import Context, Node
    F, hop = 3, 64
    node = Node(44100.0, [0])
    try:
        for B, lanes in ((1030, 16), (9, 64)):
            frames = _frames(oracle, B, F)
            ctx = Context(44100.0, solver="tree", lanes=lanes)
            try:
                assert ctx.lanes_per_utterance(B) == lanes
                ref = ctx.to_int16(ctx.synthesize(frames, hop))
            finally:
                ctx.close()
            assert np.array_equal(node.synthesize(frames, hop), ref)
    finally:
        node.close()


def test_bench_world2_gather_check_one_device():
    """bench.py's multi-process path end to end at world size 2, started as the driver starts it
    (`python bench.py --gpus 2 ...`, no torch.distributed.run in the command: bench.py starts the
    ranks), both ranks on this box's one GPU, the int16 blocks through gloo instead of RCCL: shards,
    the max-over-ranks timing, and the self-check of the exchange -- rank 0 re-synthesizes the first
    and last utterance of both blocks alone and finds the gathered rows bit for bit equal."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "1", "--batch", "24", "--seconds", "0.05",
           "--no-cpu-baseline", "--gather-transport", "gloo", "--one-device"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 48 and d["value"] > 0
    chk = d["gather_check"]
    assert chk["bitwise_equal"], chk
    assert chk["utterances_checked"] == [0, 23, 24, 47]
    assert chk["lanes_per_utterance"] == 64  # (24 utterances per rank: the voice kernel, as the shards ran)
    assert d["multi_gpu"]["transport"].startswith("gloo")
    assert d["multi_gpu"]["avg_launch_ms_max_over_ranks"] > 0
