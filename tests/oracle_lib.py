"""ctypes access to the two CHECKERS built by oracle/Makefile.

* ``Oracle``  -> oracle/_build/liboracle.so : our C restatement of the reference path.
* ``RefLib``  -> oracle/_ref/libafsref.so   : the reference's own sources + harness.

Test infrastructure only (see oracle/afs_oracle.h).  Neither library is used by the
product; tests call them to produce expected values.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from areafunctionsynthesis_amd.frames import FRAME_DTYPE

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libafsref.so")

_dp = ctypes.POINTER(ctypes.c_double)
_vp = ctypes.c_void_p


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def build_oracle() -> None:
    """Build the restatement (and the reference build when /root/reference exists)."""
    targets = ["oracle"]
    if os.path.isdir("/root/reference/src/Backend"):
        targets.append("ref")
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")] + targets)


# TdsModel::Options (TdsModel.h:83-95) in afs_options / ao_options order, with defaults
class AoOptions(ctypes.Structure):
    """ao_options (oracle/afs_oracle.h) = TdsModel::Options (TdsModel.h:83-95)."""
    _fields_ = [("turbulence_losses", ctypes.c_int), ("soft_walls", ctypes.c_int),
                ("generate_noise_sources", ctypes.c_int), ("radiation_from_skin", ctypes.c_int),
                ("piriform_fossa", ctypes.c_int), ("inner_length_corrections", ctypes.c_int),
                ("transvelar_coupling", ctypes.c_int), ("glottis_loss", ctypes.c_int), ("solver", ctypes.c_int),
                ("glottis_model", ctypes.c_int), ("flow_separation_area_ratio", ctypes.c_double)]


OPTION_DEFAULTS = {"turbulence_losses": 1, "soft_walls": 1, "generate_noise_sources": 1, "radiation_from_skin": 1,
                   "piriform_fossa": 0, "inner_length_corrections": 1, "transvelar_coupling": 0, "glottis_loss": 0,
                   "solver": 0, "glottis_model": 0, "flow_separation_area_ratio": 1.0}
OPTION_NAMES = tuple(OPTION_DEFAULTS)


def options_struct(opt: dict) -> AoOptions:
    unknown = set(opt) - set(OPTION_NAMES)
    if unknown:
        raise KeyError(f"unknown options {sorted(unknown)}")
    o = AoOptions()
    for k, d in OPTION_DEFAULTS.items():
        v = opt.get(k, d)
        setattr(o, k, float(v) if k == "flow_separation_area_ratio" else int(v))
    return o


class TargetCfg(ctypes.Structure):
    _fields_ = [("stationary_s", ctypes.c_double * 4), ("transition_s", ctypes.c_double * 3),
                ("f0_hz", ctypes.c_double * 4), ("lung_pressure_dpa", ctypes.c_double),
                ("glottis", ctypes.c_double * 6)]


class Oracle:
    """Restatement: one utterance at a time (batch 1), fp64."""

    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            build_oracle()
        lib = ctypes.CDLL(path)
        lib.ao_create.restype = _vp
        lib.ao_create.argtypes = [ctypes.c_double, ctypes.c_uint32, _vp]
        lib.ao_destroy.argtypes = [_vp]
        lib.ao_synthesize_call.restype = ctypes.c_int
        lib.ao_synthesize_call.argtypes = [_vp, _vp, ctypes.c_int, _vp]
        lib.ao_synthesize_utterance.restype = ctypes.c_long
        lib.ao_synthesize_utterance.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_uint32,
                                                ctypes.c_double, ctypes.POINTER(AoOptions), _vp]
        lib.ao_fulcher_kent.restype = ctypes.c_double
        lib.ao_fulcher_kent.argtypes = [ctypes.c_double, ctypes.c_double]
        lib.ao_get_pressures.argtypes = [_vp, _vp]
        lib.ao_get_currents.argtypes = [_vp, _vp]
        lib.ao_get_state.argtypes = [_vp, _vp, ctypes.POINTER(ctypes.c_int)]
        lib.ao_position.argtypes = [_vp]
        lib.ao_position.restype = ctypes.c_int
        lib.ao_rng_calls.argtypes = [_vp]
        lib.ao_rng_calls.restype = ctypes.c_long
        lib.ao_rng_seed.argtypes = [_vp, ctypes.c_uint32]
        lib.ao_rng_next.argtypes = [_vp]
        lib.ao_rng_next.restype = ctypes.c_int32
        lib.ao_af_to_frame.argtypes = [_vp, _vp]
        lib.ao_af_area.argtypes = [_vp, ctypes.c_double]
        lib.ao_af_area.restype = ctypes.c_double
        lib.ao_chebyshev.argtypes = [ctypes.c_double, ctypes.c_int, ctypes.c_int, _vp, _vp]
        lib.ao_chebyshev.restype = ctypes.c_int
        lib.ao_to_int16.argtypes = [_vp, ctypes.c_long, _vp]
        lib.ao_target_default.argtypes = [ctypes.POINTER(TargetCfg)]
        lib.ao_target_default.restype = None
        lib.ao_target_num_samples.argtypes = [ctypes.POINTER(TargetCfg), ctypes.c_double]
        lib.ao_target_num_samples.restype = ctypes.c_long
        lib.ao_target_frames.argtypes = [_vp, ctypes.POINTER(TargetCfg), ctypes.c_double, ctypes.c_long,
                                         ctypes.c_long, _vp]
        lib.ao_target_frames.restype = None
        self.lib = lib

    # Synthesizer::playTargetSequence ------------------------------------------
    def fulcher_kent(self, pressure_dpa: float, d_cm: float) -> float:
        return float(self.lib.ao_fulcher_kent(pressure_dpa, d_cm))

    def target_cfg(self, timing=None) -> "TargetCfg":
        c = TargetCfg()
        self.lib.ao_target_default(ctypes.byref(c))
        for k, v in (timing or {}).items():
            cur = getattr(c, k)
            if isinstance(cur, float):
                setattr(c, k, float(v))
            else:
                for i, x in enumerate(v):
                    cur[i] = float(x)
        return c

    def target_num_samples(self, fs: float, timing=None) -> int:
        return int(self.lib.ao_target_num_samples(ctypes.byref(self.target_cfg(timing)), fs))

    def target_frames(self, shapes4, fs: float, timing=None, k0: int = 0, n=None) -> np.ndarray:
        """Frames k0 .. k0+n-1 of the hop-1 trajectory (frame 0 = init() latch)."""
        c = self.target_cfg(timing)
        if n is None:
            n = int(self.lib.ao_target_num_samples(ctypes.byref(c), fs)) + 1 - k0
        s = np.ascontiguousarray(shapes4, dtype=np.float64).reshape(64)
        out = np.zeros(n, dtype=FRAME_DTYPE)
        self.lib.ao_target_frames(_ptr(s), ctypes.byref(c), fs, k0, n, _ptr(out))
        return out

    def target_sequence(self, shapes4, seed: int, fs: float, timing=None) -> np.ndarray:
        """playTargetSequence's audio: the trajectory frames played with hop 1."""
        return self.utterance(self.target_frames(shapes4, fs, timing), 1, seed, fs)

    def to_int16(self, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float64)
        out = np.zeros(x.size, dtype=np.int16)
        self.lib.ao_to_int16(_ptr(x), x.size, _ptr(out))
        return out

    def utterance(self, frames: np.ndarray, hop: int, seed: int, fs: float, opt=None) -> np.ndarray:
        """opt: dict of TdsModel options (OPTION_NAMES) overriding the defaults."""
        frames = np.ascontiguousarray(frames, dtype=FRAME_DTYPE)
        F = frames.shape[0]
        out = np.zeros((F - 1) * hop, dtype=np.float64)
        o = ctypes.byref(options_struct(opt)) if opt else None
        n = self.lib.ao_synthesize_utterance(_ptr(frames), F, hop, seed, fs, o, _ptr(out))
        assert n == out.size
        return out

    def batch(self, frames: np.ndarray, hop: int, seeds, fs: float) -> np.ndarray:
        B, F = frames.shape
        out = np.zeros((B, (F - 1) * hop), dtype=np.float64)
        for u in range(B):
            out[u] = self.utterance(frames[u], hop, int(seeds[u]), fs)
        return out

    def utterance_draws(self, frames: np.ndarray, hop: int, seed: int, fs: float):
        """(audio, rand() calls) of one utterance: the latch then F-1 calls of hop samples."""
        frames = np.ascontiguousarray(frames, dtype=FRAME_DTYPE)
        h = self.lib.ao_create(fs, seed, None)
        try:
            parts = [self.call(h, frames[k], hop) for k in range(frames.shape[0])]
            return np.concatenate(parts), int(self.lib.ao_rng_calls(h))
        finally:
            self.lib.ao_destroy(h)

    def rand_stream(self, seed: int, n: int) -> np.ndarray:
        buf = ctypes.create_string_buffer(31 * 4 + 8)
        self.lib.ao_rng_seed(buf, seed)
        return np.array([self.lib.ao_rng_next(buf) for _ in range(n)], dtype=np.int64)

    def af_to_frame(self, params16) -> np.ndarray:
        p = np.ascontiguousarray(params16, dtype=np.float64)
        f = np.zeros((), dtype=FRAME_DTYPE)
        self.lib.ao_af_to_frame(_ptr(p), f.ctypes.data_as(ctypes.c_void_p))
        return f

    def chebyshev(self, ratio: float, poles: int, highpass: bool = False):
        a = np.zeros(33)
        b = np.zeros(33)
        n = self.lib.ao_chebyshev(ratio, int(highpass), poles, _ptr(a), _ptr(b))
        return a[: n + 1], b[: n + 1]

    # step-level access -------------------------------------------------------
    def create(self, fs: float, seed: int):
        return self.lib.ao_create(fs, seed, None)

    def call(self, h, frame: np.ndarray, n: int) -> np.ndarray:
        fr = np.ascontiguousarray(frame, dtype=FRAME_DTYPE)
        out = np.zeros(max(n, 1), dtype=np.float64)
        m = self.lib.ao_synthesize_call(h, _ptr(fr), n, _ptr(out))
        return out[:m]

    def pressures(self, h) -> np.ndarray:
        p = np.zeros(93)
        self.lib.ao_get_pressures(h, _ptr(p))
        return p

    def currents(self, h) -> np.ndarray:
        u = np.zeros(97)
        self.lib.ao_get_currents(h, _ptr(u))
        return u

    def destroy(self, h) -> None:
        self.lib.ao_destroy(h)


class RefLib:
    """The reference's own classes (TdsModel, TriangularGlottis, Tube, IirFilter)."""

    def __init__(self, path: str = REF_SO):
        if not os.path.exists(path):
            build_oracle()
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        lib = ctypes.CDLL(path)
        lib.afsref_create.restype = _vp
        lib.afsref_create.argtypes = [ctypes.c_double, ctypes.c_uint]
        lib.afsref_destroy.argtypes = [_vp]
        lib.afsref_call.restype = ctypes.c_int
        lib.afsref_call.argtypes = [_vp, _vp, ctypes.c_int, _vp]
        lib.afsref_pressures.argtypes = [_vp, _vp]
        lib.afsref_currents.argtypes = [_vp, _vp]
        lib.afsref_position.argtypes = [_vp]
        lib.afsref_position.restype = ctypes.c_int
        lib.afsref_rand_calls.restype = ctypes.c_long
        lib.afsref_utterance.restype = ctypes.c_long
        lib.afsref_utterance.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_uint,
                                         ctypes.c_double, _vp]
        lib.afsref_utterance_opt.restype = ctypes.c_long
        lib.afsref_utterance_opt.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_uint,
                                             ctypes.c_double, _vp, ctypes.POINTER(AoOptions)]
        lib.afsref_fulcher_table.restype = ctypes.c_int
        lib.afsref_fulcher_table.argtypes = [ctypes.c_char_p, ctypes.c_int]
        lib.afsref_chebyshev.restype = ctypes.c_int
        lib.afsref_chebyshev.argtypes = [ctypes.c_double, ctypes.c_int, ctypes.c_int, _vp, _vp]
        lib.afsref_glibc_rand.argtypes = [ctypes.c_uint, ctypes.c_int, _vp]
        lib.afsref_to_int16.argtypes = [_vp, ctypes.c_int, _vp]
        self.lib = lib

    def fulcher_table(self) -> str:
        """stdout of TdsModel::checkGlottalEntranceLossCoeffFlucher2011 (Fulcher 2011 Table I)."""
        buf = ctypes.create_string_buffer(8192)
        n = self.lib.afsref_fulcher_table(buf, 8192)
        assert n > 0
        return buf.value.decode()

    def to_int16(self, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float64)
        out = np.zeros(x.size, dtype=np.int16)
        self.lib.afsref_to_int16(_ptr(x), x.size, _ptr(out))
        return out

    def utterance(self, frames: np.ndarray, hop: int, seed: int, fs: float, opt=None) -> np.ndarray:
        frames = np.ascontiguousarray(frames, dtype=FRAME_DTYPE)
        F = frames.shape[0]
        out = np.zeros((F - 1) * hop, dtype=np.float64)
        o = ctypes.byref(options_struct(opt or {}))
        n = self.lib.afsref_utterance_opt(_ptr(frames), F, hop, seed, fs, _ptr(out), o)
        assert n == out.size
        return out

    def batch(self, frames: np.ndarray, hop: int, seeds, fs: float) -> np.ndarray:
        B, F = frames.shape
        out = np.zeros((B, (F - 1) * hop), dtype=np.float64)
        for u in range(B):
            out[u] = self.utterance(frames[u], hop, int(seeds[u]), fs)
        return out

    def glibc_rand(self, seed: int, n: int) -> np.ndarray:
        out = np.zeros(n, dtype=np.int32)
        self.lib.afsref_glibc_rand(seed, n, _ptr(out))
        return out.astype(np.int64)

    def chebyshev(self, ratio: float, poles: int, highpass: bool = False):
        a = np.zeros(33)
        b = np.zeros(33)
        n = self.lib.afsref_chebyshev(ratio, int(highpass), poles, _ptr(a), _ptr(b))
        return a[: n + 1], b[: n + 1]

    def create(self, fs: float, seed: int):
        return self.lib.afsref_create(fs, seed)

    def call(self, h, frame: np.ndarray, n: int) -> np.ndarray:
        fr = np.ascontiguousarray(frame, dtype=FRAME_DTYPE)
        out = np.zeros(max(n, 1), dtype=np.float64)
        m = self.lib.afsref_call(h, _ptr(fr), n, _ptr(out))
        return out[:m]

    def pressures(self, h) -> np.ndarray:
        p = np.zeros(93)
        self.lib.afsref_pressures(h, _ptr(p))
        return p

    def currents(self, h) -> np.ndarray:
        u = np.zeros(97)
        self.lib.afsref_currents(h, _ptr(u))
        return u

    def destroy(self, h) -> None:
        self.lib.afsref_destroy(h)


def ref_available() -> bool:
    return os.path.exists(REF_SO) or os.path.isdir("/root/reference/src/Backend")


def _draws_job(args):
    frames, hop, seed, fs = args
    return Oracle().utterance_draws(frames, hop, seed, fs)


_MEMO = {}  # (the GPU tests compare both kernel widths with the same oracle runs)


def _memo_key(*parts) -> str:
    import hashlib
    h = hashlib.sha1()
    for p in parts:
        h.update(np.ascontiguousarray(p).tobytes() if isinstance(p, np.ndarray) else repr(p).encode())
    return h.hexdigest()


def oracle_parallel(frames: np.ndarray, hop: int, seeds, fs: float, workers: int = 0):
    """The oracle over rows of frames[B, F] in worker processes (one utterance per task).
    Returns (audio[B, T], rand() calls[B]); results are memoized per process."""
    key = _memo_key("frames", frames, int(hop), np.asarray(seeds, dtype=np.int64), float(fs))
    if key not in _MEMO:
        _MEMO[key] = _oracle_parallel(frames, hop, seeds, fs, workers)
    x, d = _MEMO[key]
    return x.copy(), d.copy()


def _oracle_parallel(frames: np.ndarray, hop: int, seeds, fs: float, workers: int = 0):
    import multiprocessing as mp
    B = frames.shape[0]
    jobs = [(np.ascontiguousarray(frames[u]), int(hop), int(seeds[u]), float(fs)) for u in range(B)]
    workers = workers or max(1, min(16, (os.cpu_count() or 1), B))
    if workers == 1:
        res = [_draws_job(j) for j in jobs]
    else:
        with mp.get_context("spawn").Pool(workers) as pool:
            res = pool.map(_draws_job, jobs)
    return np.stack([r[0] for r in res]), np.array([r[1] for r in res], dtype=np.int64)


def _target_job(args):
    shapes4, seed, fs = args
    o = Oracle()
    return o.utterance_draws(o.target_frames(shapes4, fs), 1, seed, fs)


def oracle_target_parallel(shapes4: np.ndarray, seeds, fs: float, workers: int = 0):
    """playTargetSequence in the oracle for shapes4[B, 4, 16] (the trajectory is built in each
    worker), one utterance per task.  Returns (audio[B, T], rand() calls[B]); memoized."""
    key = _memo_key("targets", shapes4, np.asarray(seeds, dtype=np.int64), float(fs))
    if key not in _MEMO:
        _MEMO[key] = _oracle_target_parallel(shapes4, seeds, fs, workers)
    x, d = _MEMO[key]
    return x.copy(), d.copy()


def _oracle_target_parallel(shapes4: np.ndarray, seeds, fs: float, workers: int = 0):
    import multiprocessing as mp
    B = shapes4.shape[0]
    jobs = [(np.ascontiguousarray(shapes4[u]), int(seeds[u]), float(fs)) for u in range(B)]
    workers = workers or max(1, min(16, (os.cpu_count() or 1), B))
    with mp.get_context("spawn").Pool(workers) as pool:
        res = pool.map(_target_job, jobs)
    return np.stack([r[0] for r in res]), np.array([r[1] for r in res], dtype=np.int64)
