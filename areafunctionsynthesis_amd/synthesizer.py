"""Host-side mirror of the reference's synthesis API on top of libafs.so.

* :class:`Context` -- one ``afs_ctx`` (device, sampling rate, solver, TdsModel options).
* :class:`Synthesizer` -- the stateful ``Synthesizer::synthesizeSignalTds`` equivalent
  (``src/Backend/Synthesizer.cpp:515-639``) for a batch of independent voices, backed by
  an ``afs_session`` whose state stays on the GPU.
* :meth:`Context.synthesize` -- whole trajectories (latch frame 0, then ``F-1`` calls of
  ``hop`` samples) for ``B`` utterances in one go.
* :meth:`Context.play_target_sequences` -- ``Synthesizer::playTargetSequence``
  (``src/Backend/Synthesizer.cpp:1299-1422``) for ``B`` utterances: four target shapes each,
  per-sample area-function tubes built on the GPU.

Arrays may be numpy arrays (host) or torch tensors on the GPU (device pointers are
passed straight to the library).
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from . import _native
from .frames import FRAME_DTYPE

_vp = ctypes.c_void_p

SOLVERS = {"cholesky": _native.AFS_SOLVER_CHOLESKY, "tree": _native.AFS_SOLVER_TREE, "sor": _native.AFS_SOLVER_SOR}


def _addr(x) -> int:
    if x is None:
        return 0
    if hasattr(x, "data_ptr"):
        return int(x.data_ptr())
    if isinstance(x, np.ndarray):
        if not x.flags["C_CONTIGUOUS"]:
            raise ValueError("array must be C-contiguous")
        return int(x.ctypes.data)
    raise TypeError(f"unsupported buffer type {type(x)}")


def _nbytes(x) -> int:
    if hasattr(x, "element_size"):
        return int(x.numel() * x.element_size())
    return int(x.nbytes)


class Context:
    """An afs_ctx: device + sampling rate + solver + options (TdsModel::Options)."""

    def __init__(self, sampling_rate_hz: float = 22050.0, solver: str = "tree", device: int = 0,
                 async_calls: bool = False, profile: bool = False, lanes: Optional[int] = None, **options):
        """``lanes``: tree solver, lanes per utterance (16: the throughput kernel, 64: the voice
        kernel); None lets the library pick per batch (AFS_LANES_16 / AFS_LANES_64, afs.h)."""
        lib = _native.load()
        cfg = _native.AfsConfig()
        lib.afs_config_default(ctypes.byref(cfg))
        cfg.sampling_rate_hz = float(sampling_rate_hz)
        cfg.solver = SOLVERS[solver]
        cfg.device = int(device)
        cfg.flags = (_native.AFS_ASYNC if async_calls else 0) | (_native.AFS_PROFILE if profile else 0)
        if lanes is not None:
            cfg.flags |= {16: _native.AFS_LANES_16, 64: _native.AFS_LANES_64}[int(lanes)]
        for k, v in options.items():
            if not hasattr(cfg.options, k):
                raise TypeError(f"unknown option {k}")
            if k == "flow_separation_area_ratio":
                setattr(cfg.options, k, float(v))
            elif k in ("glottis_loss", "glottis_model"):
                setattr(cfg.options, k, int(v))
            else:
                setattr(cfg.options, k, int(bool(v)))
        h = _vp()
        _native.check(lib.afs_create(ctypes.byref(h), ctypes.byref(cfg)), None, "afs_create")
        self._lib = lib
        self._h = h
        self.sampling_rate_hz = float(sampling_rate_hz)
        self.solver = solver
        self.device = int(device)

    @property
    def handle(self):
        return self._h

    def close(self) -> None:
        if self._h:
            self._lib.afs_destroy(self._h)
            self._h = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def lanes_per_utterance(self, batch: int) -> int:
        """Lanes per utterance the tree solver uses for a batch of this size."""
        return int(self._lib.afs_lanes_per_utterance(self._h, int(batch)))

    def synthesis_kernel(self, batch: int) -> str:
        """Name of the synthesis kernel a batch of this size runs (for matching profiler output)."""
        return self._lib.afs_synthesis_kernel(self._h, int(batch)).decode()

    def set_stream(self, stream_handle: int) -> None:
        """Issue all work on this hipStream_t (e.g. torch.cuda.current_stream().cuda_stream)."""
        _native.check(self._lib.afs_set_stream(self._h, _vp(stream_handle)), self._h, "afs_set_stream")

    def synchronize(self) -> None:
        _native.check(self._lib.afs_synchronize(self._h), self._h, "afs_synchronize")

    def synthesize(self, frames, hop: int, seeds=None, out=None, report: bool = False, nonfinite=None):
        """frames[B, F] (FRAME_DTYPE array, or a uint8 torch tensor [B, F, 1072] on the GPU)
        -> audio[B, (F-1)*hop] float64.  ``seeds=None``: 1 .. B.  ``nonfinite``: optional uint8
        array / tensor of B flags (1 = the utterance's audio holds NaN/Inf); with ``report``
        the returned dict carries them under ``nonfinite`` too."""
        if isinstance(frames, np.ndarray):
            if frames.dtype != FRAME_DTYPE or frames.ndim != 2:
                raise ValueError("frames must be a 2-D FRAME_DTYPE array [B, F]")
            B, F = frames.shape
            frames = np.ascontiguousarray(frames)
        else:
            B, F = int(frames.shape[0]), int(frames.shape[1])
            if _nbytes(frames) != B * F * FRAME_DTYPE.itemsize:
                raise ValueError("device frames must hold B*F*1072 bytes")
        T = (F - 1) * hop
        if seeds is None:
            seeds = np.arange(1, B + 1, dtype=np.uint32)
        if isinstance(seeds, np.ndarray):
            seeds = np.ascontiguousarray(seeds, dtype=np.uint32)
        if out is None:
            out = np.zeros((B, T), dtype=np.float64)
        if _nbytes(out) != B * T * 8:
            raise ValueError("out must hold B*(F-1)*hop doubles")
        if nonfinite is None and report:
            nonfinite = np.zeros(B, dtype=np.uint8)
        if nonfinite is not None and _nbytes(nonfinite) != B:
            raise ValueError("nonfinite must hold B bytes")
        # (a report makes the call wait for the device: only when asked, so that an AFS_ASYNC context's
        # calls with device buffers return once queued)
        rep = _native.AfsReport()
        st = self._lib.afs_synthesize(self._h, _vp(_addr(frames)), _vp(_addr(seeds)), B, F, hop,
                                      _vp(_addr(out)), _vp(_addr(nonfinite)), ctypes.byref(rep) if report else None)
        _native.check(st, self._h, "afs_synthesize")
        if report:
            return out, {"device_ms": rep.device_ms, "samples": rep.samples,
                         "nonfinite_utterances": rep.nonfinite_utterances, "kernel": rep.kernel,
                         "nonfinite": nonfinite}
        return out

    def noise_plans(self, frames: np.ndarray, hop: int, s_begin: int = 0, s_end: Optional[int] = None) -> np.ndarray:
        """Diagnostics (tree solver): the noise-source plan records K5 computes for samples
        [s_begin, s_end) of frames[rows, F] -> uint64[rows, s_end - s_begin, AFS_PLAN_WORDS]."""
        if frames.dtype != FRAME_DTYPE or frames.ndim != 2:
            raise ValueError("frames must be a 2-D FRAME_DTYPE array [rows, F]")
        rows, F = frames.shape
        if s_end is None:
            s_end = (F - 1) * hop
        frames = np.ascontiguousarray(frames)
        out = np.zeros((rows, s_end - s_begin, _native.AFS_PLAN_WORDS), dtype=np.uint64)
        st = self._lib.afs_noise_plans(self._h, _vp(_addr(frames)), rows, F, hop, s_begin, s_end, _vp(_addr(out)))
        _native.check(st, self._h, "afs_noise_plans")
        return out

    def noise_plan_hops(self, frames: np.ndarray, hop: int, s_begin: int = 0, s_end: Optional[int] = None):
        """Diagnostics (tree solver, hop >= AFS_PLAN_HOP_MIN): K5's hop records of the hops samples
        [s_begin, s_end) span -> (uint8[rows, slots, AFS_PLAN_HOP_BYTES], the dense records of the
        mixed hops' samples uint64[rows, s_end - s_begin, AFS_PLAN_WORDS], zero elsewhere)."""
        if frames.dtype != FRAME_DTYPE or frames.ndim != 2:
            raise ValueError("frames must be a 2-D FRAME_DTYPE array [rows, F]")
        rows, F = frames.shape
        if s_end is None:
            s_end = (F - 1) * hop
        frames = np.ascontiguousarray(frames)
        slots = (s_end - 1) // hop - s_begin // hop + 1
        hops = np.zeros((rows, slots, _native.AFS_PLAN_HOP_BYTES), dtype=np.uint8)
        plans = np.zeros((rows, s_end - s_begin, _native.AFS_PLAN_WORDS), dtype=np.uint64)
        st = self._lib.afs_noise_plan_hops(self._h, _vp(_addr(frames)), rows, F, hop, s_begin, s_end,
                                           _vp(_addr(hops)), _vp(_addr(plans)))
        _native.check(st, self._h, "afs_noise_plan_hops")
        return hops, plans

    def plan_hop_words(self, hops: np.ndarray, ratio: np.ndarray) -> np.ndarray:
        """Diagnostics (tree solver): the plan words the synthesis kernel evaluates per sample from
        hop records hops[n, AFS_PLAN_HOP_BYTES] (uint8) at ratio[n] -> uint64[n, AFS_PLAN_WORDS]."""
        hops = np.ascontiguousarray(hops, dtype=np.uint8)
        ratio = np.ascontiguousarray(ratio, dtype=np.float64)
        n = ratio.shape[0]
        if hops.shape != (n, _native.AFS_PLAN_HOP_BYTES):
            raise ValueError("hops must be uint8[n, AFS_PLAN_HOP_BYTES]")
        out = np.zeros((n, _native.AFS_PLAN_WORDS), dtype=np.uint64)
        st = self._lib.afs_plan_hop_words(self._h, _vp(_addr(hops)), _vp(_addr(ratio)), n, _vp(_addr(out)))
        _native.check(st, self._h, "afs_plan_hop_words")
        return out

    def tube_interpolate(self, left: np.ndarray, right: np.ndarray, ratio: np.ndarray):
        """Diagnostics (tree solver): the synthesis kernel's interpolated pharynx/mouth areas and
        lengths for frames left[n], right[n] at ratio[n] -> (area[n, 40], length[n, 40])."""
        left = np.ascontiguousarray(left, dtype=FRAME_DTYPE)
        right = np.ascontiguousarray(right, dtype=FRAME_DTYPE)
        ratio = np.ascontiguousarray(ratio, dtype=np.float64)
        n = ratio.shape[0]
        if left.shape != (n,) or right.shape != (n,):
            raise ValueError("left, right and ratio must have n entries")
        area = np.zeros((n, 40))
        length = np.zeros((n, 40))
        st = self._lib.afs_tube_interpolate(self._h, _vp(_addr(left)), _vp(_addr(right)), _vp(_addr(ratio)), n,
                                            _vp(_addr(area)), _vp(_addr(length)))
        _native.check(st, self._h, "afs_tube_interpolate")
        return area, length

    def kernel_times(self) -> dict:
        """(profile=True contexts) summed device time and count of the synthesis-kernel (K1),
        noise-source-plan (K5) and output-stage (K6) launches since the previous call (waits for
        the stream)."""
        t = _native.AfsKernelTiming()
        _native.check(self._lib.afs_kernel_times_ex(self._h, ctypes.byref(t)), self._h, "afs_kernel_times_ex")
        return {"synth_ms": t.synth_ms, "synth_launches": t.synth_launches, "plan_ms": t.plan_ms,
                "plan_launches": t.plan_launches, "output_ms": t.output_ms, "output_launches": t.output_launches}

    def rng_draws(self, batch: int) -> np.ndarray:
        """rand() calls per utterance of the last synthesize / play_target_sequences call
        (tree solver; the reference's count is what a wrapped rand() would count)."""
        d = np.zeros(int(batch), dtype=np.int64)
        _native.check(self._lib.afs_rng_draws(self._h, int(batch), _vp(_addr(d))), self._h, "afs_rng_draws")
        return d

    def af_to_frames(self, params, frames=None):
        """OneDimAreaFunction::calculateOneDimTubeFunction on the GPU.
        params[..., 16] -> frames[...] (tube fields filled; velum/glottis left as given)."""
        p = np.ascontiguousarray(params, dtype=np.float64)
        shape = p.shape[:-1]
        n = int(np.prod(shape)) if shape else 1
        if frames is None:
            frames = np.zeros(shape, dtype=FRAME_DTYPE)
        st = self._lib.afs_af_to_frames(self._h, _vp(_addr(p)), n, _vp(_addr(frames)))
        _native.check(st, self._h, "afs_af_to_frames")
        return frames


    def target_sequence_samples(self, timing: Optional[dict] = None) -> int:
        """numSamples of playTargetSequence (``SAMPLING_RATE * totalTime_s``, truncated)."""
        ts = target_sequence(timing)
        return int(self._lib.afs_target_sequence_samples(ctypes.byref(ts), self.sampling_rate_hz))

    def play_target_sequences(self, shapes, targets, timing: Optional[dict] = None, seeds=None, out=None,
                              report: bool = False):
        """``playTargetSequence(targetShape, stationary_s, transition_s)`` for every row of
        ``targets[B, 4]`` (indices into ``shapes[S, 16]``) -> audio[B, T] float64.

        ``timing`` overrides fields of :func:`target_sequence` (``stationary_s``,
        ``transition_s``, ``f0_hz``, ``lung_pressure_dpa``, ``glottis``)."""
        shapes = np.ascontiguousarray(shapes, dtype=np.float64)
        targets = np.ascontiguousarray(targets, dtype=np.int32)
        if shapes.ndim != 2 or shapes.shape[1] != 16 or targets.ndim != 2 or targets.shape[1] != 4:
            raise ValueError("shapes must be [S, 16] and targets [B, 4]")
        ts = target_sequence(timing)
        B = targets.shape[0]
        T = int(self._lib.afs_target_sequence_samples(ctypes.byref(ts), self.sampling_rate_hz))
        if T < 0:
            raise ValueError("bad target-sequence timing")
        if seeds is None:
            seeds = np.arange(1, B + 1, dtype=np.uint32)
        if isinstance(seeds, np.ndarray):
            seeds = np.ascontiguousarray(seeds, dtype=np.uint32)
        if out is None:
            out = np.zeros((B, T), dtype=np.float64)
        if _nbytes(out) != B * T * 8:
            raise ValueError("out must hold B*T doubles")
        nonfinite = np.zeros(B, dtype=np.uint8) if report else None
        rep = _native.AfsReport()
        st = self._lib.afs_play_target_sequences(self._h, _vp(_addr(shapes)), shapes.shape[0], _vp(_addr(targets)),
                                                 ctypes.byref(ts), _vp(_addr(seeds)), B, _vp(_addr(out)),
                                                 _vp(_addr(nonfinite)), ctypes.byref(rep))
        _native.check(st, self._h, "afs_play_target_sequences")
        if report:
            return out, {"device_ms": rep.device_ms, "samples": rep.samples,
                         "nonfinite_utterances": rep.nonfinite_utterances, "nonfinite": nonfinite}
        return out

    def to_int16(self, samples, out=None):
        """The reference's int16 audio ring format (Synthesizer.cpp:955-973) on the GPU:
        short(x * 32767) truncated, clipped outside [-1, 1], NaN -> 0."""
        if isinstance(samples, np.ndarray):
            samples = np.ascontiguousarray(samples, dtype=np.float64)
            n = samples.size
            if out is None:
                out = np.zeros(samples.shape, dtype=np.int16)
        else:
            n = int(samples.numel())
            if out is None:
                import torch
                out = torch.empty(tuple(samples.shape), dtype=torch.int16, device=samples.device)
        if _nbytes(out) != n * 2:
            raise ValueError("out must hold one int16 per sample")
        st = self._lib.afs_to_int16(self._h, _vp(_addr(samples)), n, _vp(_addr(out)))
        _native.check(st, self._h, "afs_to_int16")
        return out


def shard_range(total: int, world: int, rank: int):
    """afs_shard_range: (first, count) of ``rank``'s contiguous block of ``total`` utterances."""
    f, n = ctypes.c_int64(), ctypes.c_int64()
    _native.load().afs_shard_range(int(total), int(world), int(rank), ctypes.byref(f), ctypes.byref(n))
    return f.value, n.value


def comm_unique_id() -> bytes:
    """afs_comm_unique_id (rank 0): the RCCL id every rank passes to :class:`Comm`."""
    buf = (ctypes.c_uint8 * _native.AFS_COMM_ID_BYTES)()
    _native.check(_native.load().afs_comm_unique_id(buf), None, "afs_comm_unique_id")
    return bytes(buf)


class Comm:
    """afs_comm: this process's rank of the audio gather (one process per GPU, RCCL)."""

    def __init__(self, ctx: Context, uid: bytes, rank: int, world: int):
        if len(uid) != _native.AFS_COMM_ID_BYTES:
            raise ValueError("the unique id holds AFS_COMM_ID_BYTES bytes")
        self.ctx, self.rank, self.world = ctx, int(rank), int(world)
        buf = (ctypes.c_uint8 * _native.AFS_COMM_ID_BYTES).from_buffer_copy(uid)
        h = _vp()
        _native.check(ctx._lib.afs_comm_create(ctx.handle, buf, self.rank, self.world, ctypes.byref(h)), ctx.handle,
                      "afs_comm_create")
        self._h, self._lib = h, ctx._lib

    def gather_pcm(self, local, root_out=None, root_counts=None) -> None:
        """afs_gather_pcm: int16 device tensor ``local`` to rank 0's ``root_out`` (device)."""
        counts = None
        if root_counts is not None:
            counts = np.ascontiguousarray(root_counts, dtype=np.int64)
        n = int(local.numel()) if hasattr(local, "numel") else int(local.size)
        _native.check(self._lib.afs_gather_pcm(self._h, _vp(_addr(local)), n, _vp(_addr(root_out)),
                                               _vp(_addr(counts))), self.ctx.handle, "afs_gather_pcm")

    def fence(self) -> None:
        _native.check(self._lib.afs_comm_fence(self._h), self.ctx.handle, "afs_comm_fence")

    def synchronize(self) -> None:
        _native.check(self._lib.afs_comm_synchronize(self._h), self.ctx.handle, "afs_comm_synchronize")

    def gather_times(self) -> dict:
        """afs_comm_gather_times: device time and count of this rank's gathers since the last call
        (HIP events on the comm's stream; waits for it)."""
        ms, n = ctypes.c_double(), ctypes.c_int32()
        _native.check(self._lib.afs_comm_gather_times(self._h, ctypes.byref(ms), ctypes.byref(n)), self.ctx.handle,
                      "afs_comm_gather_times")
        return {"gather_ms": ms.value, "gathers": n.value}

    def close(self) -> None:
        if self._h:
            self._lib.afs_comm_destroy(self._h)
            self._h = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Node:
    """Several GPUs driven from this one process (afs_comm_create_all + afs_multi_synthesize):
    ``synthesize`` shards the batch over the devices and returns the int16 audio of the whole
    batch, gathered to the first device over RCCL."""

    def __init__(self, sampling_rate_hz: float, devices: Sequence[int], solver: str = "tree", **options):
        self.ctxs = [Context(sampling_rate_hz, solver=solver, device=d, **options) for d in devices]
        n = len(self.ctxs)
        hs = (_vp * n)(*[c.handle for c in self.ctxs])
        self._comms = (_vp * n)()
        lib = self.ctxs[0]._lib
        _native.check(lib.afs_comm_create_all(hs, n, self._comms), self.ctxs[0].handle, "afs_comm_create_all")
        self._hs, self._lib = hs, lib

    def synthesize(self, frames: np.ndarray, hop: int, seeds=None, pcm_out=None, report: bool = False):
        frames = np.ascontiguousarray(frames, dtype=FRAME_DTYPE)
        B, F = frames.shape
        T = (F - 1) * hop
        if seeds is not None:
            seeds = np.ascontiguousarray(seeds, dtype=np.uint32)
        if pcm_out is None:
            pcm_out = np.zeros((B, T), dtype=np.int16)
        nonfinite = np.zeros(B, dtype=np.uint8)
        rep = _native.AfsReport()
        st = self._lib.afs_multi_synthesize(self._hs, self._comms, len(self.ctxs), _vp(_addr(frames)),
                                            _vp(_addr(seeds)), B, F, hop, _vp(_addr(pcm_out)), _vp(_addr(nonfinite)),
                                            ctypes.byref(rep))
        _native.check(st, self.ctxs[0].handle, "afs_multi_synthesize")
        if report:
            return pcm_out, {"device_ms": rep.device_ms, "samples": rep.samples,
                             "nonfinite_utterances": rep.nonfinite_utterances, "nonfinite": nonfinite}
        return pcm_out

    def close(self) -> None:
        for i in range(len(self.ctxs)):
            if self._comms[i]:
                self._lib.afs_comm_destroy(self._comms[i])
                self._comms[i] = None
        for c in self.ctxs:
            c.close()


def target_sequence(overrides: Optional[dict] = None) -> "_native.AfsTargetSequence":
    """afs_target_sequence with the reference's constants (afs_target_sequence_default) and
    the given fields replaced."""
    ts = _native.AfsTargetSequence()
    _native.load().afs_target_sequence_default(ctypes.byref(ts))
    for k, v in (overrides or {}).items():
        if not hasattr(ts, k):
            raise TypeError(f"unknown target-sequence field {k}")
        cur = getattr(ts, k)
        if isinstance(cur, float):
            setattr(ts, k, float(v))
        else:
            vals = list(v)
            if len(vals) != len(cur):
                raise ValueError(f"{k} takes {len(cur)} values")
            for i, x in enumerate(vals):
                cur[i] = float(x)
    return ts


class Synthesizer:
    """Batch of ``B`` voices with the reference's incremental synthesis semantics.

    ``synthesize_signal_tds(frames, n)`` is ``Synthesizer::synthesizeSignalTds(newTube,
    newGlottisParams, n, newSignal)`` applied to every voice: the first call after
    construction / :meth:`reset` only latches the frames and returns an empty array.
    """

    def __init__(self, context: Context, batch: int = 1, seeds: Optional[Sequence[int]] = None):
        self.ctx = context
        self.batch = int(batch)
        lib = context._lib
        s = np.arange(1, self.batch + 1, dtype=np.uint32) if seeds is None else np.asarray(seeds, dtype=np.uint32)
        h = _vp()
        _native.check(lib.afs_session_create(context.handle, self.batch, _vp(_addr(s)), ctypes.byref(h)),
                      context.handle, "afs_session_create")
        self._h = h
        self._lib = lib

    def reset(self, seeds: Optional[Sequence[int]] = None) -> None:
        s = np.arange(1, self.batch + 1, dtype=np.uint32) if seeds is None else np.asarray(seeds, dtype=np.uint32)
        _native.check(self._lib.afs_session_reset(self._h, _vp(_addr(s))), self.ctx.handle, "afs_session_reset")

    def synthesize_signal_tds(self, frames: np.ndarray, num_samples: int) -> np.ndarray:
        fr = np.ascontiguousarray(np.broadcast_to(frames, (self.batch,)), dtype=FRAME_DTYPE)
        n = max(int(num_samples), 1)
        out = np.zeros((self.batch, n), dtype=np.float64)
        produced = ctypes.c_int32(0)
        st = self._lib.afs_session_synthesize(self._h, _vp(_addr(fr)), int(num_samples), _vp(_addr(out)), None,
                                              ctypes.byref(produced), None)
        _native.check(st, self.ctx.handle, "afs_session_synthesize")
        return out[:, : produced.value]

    def rng_draws(self) -> np.ndarray:
        """rand() calls of every voice since construction / the last reset (tree solver)."""
        d = np.zeros(self.batch, dtype=np.int64)
        _native.check(self._lib.afs_session_rng_draws(self._h, _vp(_addr(d))), self.ctx.handle,
                      "afs_session_rng_draws")
        return d

    # reference spelling
    synthesizeSignalTds = synthesize_signal_tds

    def close(self) -> None:
        if self._h:
            self._lib.afs_session_destroy(self._h)
            self._h = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
