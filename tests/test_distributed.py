"""Multi-process path of bench.py on CPU (gloo, world size 2): shards cover the batch
exactly once, rank-local workloads equal the rows of the full batch, seeds are the global
u + 1, and the gather reassembles the audio in utterance order.  The synthesis on each rank is
the tree kernel's own phase code run on the CPU (tests/emu: the host build of tree_core.h, the
code the GPU kernel executes lane by lane), so the gathered audio is real synthesized audio,
checked against a single-process run of the whole batch and against the oracle."""
import ctypes
import os
import socket
import subprocess

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from areafunctionsynthesis_amd import sharding, workloads

B, SECONDS, FS = 6, 0.03, 44100.0


EMU = os.path.join(os.path.dirname(os.path.abspath(__file__)), "emu")


def _frames(w):
    from oracle_lib import Oracle
    orc = Oracle()
    return workloads.build_frames(w, lambda p: np.stack([orc.af_to_frame(r) for r in p]))


def _synth(w) -> torch.Tensor:
    """[B, T] float64: the rank's utterances synthesized by the tree kernel's phase code on the
    CPU (tests/emu/tree_emu.cpp, 16 lanes per utterance as on the GPU)."""
    from areafunctionsynthesis_amd.frames import FRAME_DTYPE
    lib = ctypes.CDLL(os.path.join(EMU, "libtree_emu.so"))
    vp = ctypes.c_void_p
    lib.emu_tree_utterance.restype = ctypes.c_long
    lib.emu_tree_utterance.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_double,
                                       ctypes.c_int, vp, vp, vp, ctypes.c_int]
    frames = _frames(w)
    out = np.zeros((w.batch, w.samples_per_utterance))
    dummy = np.zeros(97)
    for u in range(w.batch):
        fr = np.ascontiguousarray(frames[u], dtype=FRAME_DTYPE)
        o = np.zeros(out.shape[1])
        n = lib.emu_tree_utterance(fr.ctypes.data, fr.size, w.hop, int(w.seeds[u]), w.fs, 16, o.ctypes.data,
                                   dummy.ctypes.data, dummy.ctypes.data, 0)
        assert n == o.size
        out[u] = o
    return torch.from_numpy(out)


def _to_int16(x: torch.Tensor, out: torch.Tensor) -> None:
    """CPU stand-in for Context.to_int16 (the oracle's restatement of the int16 stage)."""
    from oracle_lib import Oracle
    out.copy_(torch.from_numpy(Oracle().to_int16(x.numpy())).reshape(out.shape))


def _resynth_int16(us):
    """The global utterances `us` synthesized alone (one-utterance workloads at index u, seed u + 1)
    and converted to int16: what bench.py's rank 0 recomputes for the gather check."""
    ws = [workloads.static_vowels(1, seconds=SECONDS, fs=FS, first_utterance=u) for u in us]
    x = torch.cat([_synth(w) for w in ws])
    o = torch.empty(x.shape, dtype=torch.int16)
    _to_int16(x, o)
    return o.numpy()


def test_gather_check_reports_a_corrupt_row():
    """check_gathered flags a gathered row that differs from the re-synthesized utterance (the
    check has teeth), and names it."""
    world, n, T = 3, 4, 50
    rng = np.random.default_rng(1)
    full = rng.integers(-32768, 32767, size=(world * n, T)).astype(np.int16)
    edges = sharding.edge_utterances(world, n)
    assert [u for _, _, u in edges] == [0, 3, 4, 7, 8, 11]
    rows = np.stack([full[u] for _, _, u in edges])
    ok = sharding.check_gathered(rows, world, n, lambda us: full[list(us)])
    assert ok["bitwise_equal"] and not ok["mismatches"]
    rows[3, 17] ^= 1  # rank 1's last row
    bad = sharding.check_gathered(rows, world, n, lambda us: full[list(us)])
    assert not bad["bitwise_equal"]
    assert bad["mismatches"] == [{"utterance": 7, "rank": 1, "row": 3, "differing_samples": 1}]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, n = sharding.shard_range(rank, world, B)
    w = workloads.static_vowels(n, seconds=SECONDS, fs=FS, first_utterance=first)
    out = _synth(w)
    got = sharding.gather_to_rank0(out, world, rank, dist)
    pcm = []
    pg = sharding.PcmGather(_to_int16, out.shape, world, rank, sharding.TorchTransport(dist, world, rank), depth=2)
    for scale in (0.5, -3.0, 1.0):  # three steps through two rotating buffers
        slot = pg.submit(torch.sin(out * 1e3) * scale)
        if slot == 1 or scale == 1.0:
            pg.drain()
            if rank == 0:
                pcm.append(pg.result(slot).reshape(-1, out.shape[1]).numpy().copy())
    # bench.py's self-check of the exchange: the synthesized audio itself through the gather, then
    # rank 0 re-synthesizes the edge utterances of every block alone and compares bit for bit
    slot = pg.submit(out)
    pg.drain()
    check = None
    if rank == 0:
        root = pg.result(slot)
        rows = torch.stack([root[r, j] for r, j, _ in sharding.edge_utterances(world, n)])
        check = sharding.check_gathered(rows, world, n, _resynth_int16)
    t = torch.tensor([float(out.numel())], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # the bench's max-over-ranks timing reduction
    if rank == 0:
        q.put((torch.cat(got).numpy(), w.seeds.copy(), float(t.item()), pcm, check))
    else:
        q.put(("seeds", w.seeds.copy()))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range():
    assert sharding.shard_range(0, 2, 5) == (0, 5)
    assert sharding.shard_range(1, 2, 5) == (5, 5)
    with pytest.raises(ValueError):
        sharding.shard_range(2, 2, 5)


def test_gloo_world2_gather_matches_single_process():
    world = 2
    subprocess.check_call(["make", "-s", "-C", EMU])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    gathered = next(r for r in res if not isinstance(r[0], str))
    audio, seeds0, numel, pcm, check = gathered
    assert check["bitwise_equal"], check
    assert check["utterances_checked"] == [0, B - 1, B, 2 * B - 1]
    seeds1 = next(r[1] for r in res if isinstance(r[0], str))
    full = workloads.static_vowels(world * B, seconds=SECONDS, fs=FS)
    ref = _synth(full).numpy()
    assert np.array_equal(audio, ref)
    from oracle_lib import Oracle
    fr = _frames(full)
    for u in (0, B - 1, B, 2 * B - 1):  # shard edges: the oracle on the same frames and seeds
        y = Oracle().utterance(fr[u], full.hop, int(full.seeds[u]), FS)
        assert np.abs(audio[u] - y).max() <= 1e-9, u
    assert np.array_equal(np.concatenate([seeds0, seeds1]), np.arange(1, world * B + 1, dtype=np.uint32))
    assert numel == B * full.samples_per_utterance
    x = np.sin(ref * 1e3)
    assert len(pcm) == 2
    assert np.array_equal(pcm[0], Oracle().to_int16(x * -3.0).reshape(x.shape))  # step 2 (slot 1)
    assert np.array_equal(pcm[1], Oracle().to_int16(x).reshape(x.shape))  # step 3 reused slot 0


def test_shard_gather_loopback(tmp_path):
    """afs_gather.h -- the shard and gather logic libafs.so drives over RCCL -- over an
    in-process loopback transport (one thread per rank): uneven shards, world 1..8, built with
    AddressSanitizer and UndefinedBehaviorSanitizer."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "gather_main")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-pthread",
                           "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                           "-I", os.path.join(root, "areafunctionsynthesis_amd", "csrc"),
                           os.path.join(root, "tests", "cpp", "gather_main.cpp"), "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout
    assert out.strip() == "gather-ok"


def test_library_shard_range_matches():
    """afs_shard_range (the C ABI export) partitions exactly like afs_gather.h."""
    from areafunctionsynthesis_amd.synthesizer import shard_range
    for total, world in ((65536, 8), (10, 3), (7, 8), (0, 2)):
        nxt = 0
        for r in range(world):
            f, n = shard_range(total, world, r)
            assert f == nxt
            nxt += n
            assert n in (total // world, total // world + 1)
        assert nxt == total
    assert shard_range(65536, 8, 3) == (3 * 8192, 8192)
