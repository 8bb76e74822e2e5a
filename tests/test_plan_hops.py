"""CPU checks of the noise-source plan's hop mode (csrc/tree_plan.h, K5 in tds_plan.hip): the
interval evaluation that decides a whole hop at once never disagrees with the per-sample
decisions, and the words a hop record yields equal the per-sample records (the discrete words
and the area terms bit for bit, the downstream factors within 1e-12 and the glottis gain within
1e-13 relative).

The host functions are the ones the GPU kernels run (the same header compiled for the CPU, test
build tests/emu); tests/test_plan_gpu.py compares the GPU's hop records with them."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from areafunctionsynthesis_amd import workloads
from areafunctionsynthesis_amd.frames import DEFAULT_GLOTTIS, FRAME_DTYPE
from areafunctionsynthesis_amd.params import default_shapes

EMU = os.path.join(os.path.dirname(os.path.abspath(__file__)), "emu")
PLAN_WORDS = 16
HOP_DTYPE = np.dtype([("p", "<f8", (PLAN_WORDS, 4)), ("kind", "u1", (PLAN_WORDS,)), ("mixed", "<u4"),
                      ("dense", "<u4"), ("noise", "<u8")])
PW_FDN, PW_GAIN_G = 3, 15


@pytest.fixture(scope="module")
def lib():
    subprocess.check_call(["make", "-s", "-C", EMU])
    lib = ctypes.CDLL(os.path.join(EMU, "libplan_emu.so"))
    vp = ctypes.c_void_p
    lib.emu_plan_iv_check.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long, ctypes.c_long, vp]
    lib.emu_plan_hops.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long, ctypes.c_long,
                                  ctypes.c_double, ctypes.c_int, vp]
    lib.emu_plan_records.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long, ctypes.c_long,
                                     ctypes.c_double, ctypes.c_int, vp]
    lib.emu_plan_hop_words.argtypes = [vp, ctypes.c_double, vp]
    return lib


def _frames(oracle, w):
    return np.ascontiguousarray(workloads.build_frames(w, lambda p: np.stack([oracle.af_to_frame(r) for r in p])))


def _shape_walk(oracle, n_rows=24, F=6, seed=3):
    """Transitions between all Default.params shapes, velum and laterality varied."""
    sh = default_shapes()
    names = sorted(sh)
    rng = np.random.default_rng(seed)
    rows = []
    for k in range(n_rows):
        fr = np.stack([oracle.af_to_frame(sh[names[int(rng.integers(len(names)))]]) for _ in range(F)])
        fr["glottis"] = DEFAULT_GLOTTIS
        fr["velum_opening_cm2"] = rng.random(F) * (k % 2)
        fr["laterality"][:, 28:36] = 0.3 * rng.random((F, 8)) * (k % 3 == 0)
        rows.append(fr)
    return np.ascontiguousarray(np.stack(rows).astype(FRAME_DTYPE))


def _cases(oracle):
    yield "static vowels", _frames(oracle, workloads.static_vowels(48, seconds=0.05, fs=44100.0)), 441
    yield "fricatives", _frames(oracle, workloads.fricatives(48, seconds=0.05, fs=44100.0, velum_cm2=1.0)), 441
    yield "frame-rate VCV", _frames(oracle, workloads.vcv(24, fs=44100.0)), 441
    yield "shape walk", _shape_walk(oracle), 97


def test_interval_decisions_never_disagree(lib, oracle):
    """Every hop the interval evaluation decides gives all its samples the decisions plan_decide
    makes on each sample (0 violations); the rest go to the per-sample path."""
    for label, frames, hop in _cases(oracle):
        rows, F = frames.shape
        n = (F - 1) * hop
        for s0, s1 in ((0, n), (hop // 3, n - hop // 2)):  # whole utterances; ranges cut inside hops
            c = np.zeros(4, dtype=np.int64)
            assert lib.emu_plan_iv_check(frames.ctypes.data, rows, F, hop, s0, s1, c.ctypes.data) == 0
            decided, undecided, violations, mixed = (int(v) for v in c)
            assert violations == 0, (label, s0, s1)
            assert mixed <= undecided, label  # a hop whose decisions change is never "decided"
            if label in ("static vowels", "fricatives"):
                assert decided >= 0.8 * (decided + undecided), (label, decided, undecided)


def test_hop_record_words_equal_dense_records(lib, oracle):
    """The words of a (not mixed) hop record, evaluated at each sample, against the dense
    per-sample record: discrete words and area terms bit for bit, downstream factors and the
    glottis gain within 1e-12 (absolute: the factors are weights in [0, 1], ratios of
    interpolated end values instead of sequential position sums, whose difference cancels) and
    1e-13 (relative)."""
    for label, frames, hop in _cases(oracle):
        rows, F = frames.shape
        n = (F - 1) * hop
        hops = np.zeros((rows, F - 1), dtype=HOP_DTYPE)
        assert lib.emu_plan_hops(frames.ctypes.data, rows, F, hop, 0, n, 44100.0, 0, hops.ctypes.data) == 0
        dense = np.zeros((rows, n, PLAN_WORDS), dtype=np.uint64)
        assert lib.emu_plan_records(frames.ctypes.data, rows, F, hop, 0, n, 44100.0, 0, dense.ctypes.data) == 0
        checked = 0
        for r in range(rows):
            for q in range(F - 1):
                h = hops[r, q]
                if h["mixed"]:
                    continue
                for i in range(0, hop, 7):
                    w = np.zeros(PLAN_WORDS, dtype=np.uint64)
                    hc = np.ascontiguousarray(h)
                    lib.emu_plan_hop_words(hc.ctypes.data, i / hop, w.ctypes.data)
                    d = dense[r, q * hop + i]
                    exact = np.ones(PLAN_WORDS, dtype=bool)
                    exact[PW_FDN:PW_FDN + 4] = False
                    exact[PW_GAIN_G] = False
                    assert np.array_equal(w[exact], d[exact]), (label, r, q, i)
                    fw, fd = w[PW_FDN:PW_FDN + 4].view(np.float64), d[PW_FDN:PW_FDN + 4].view(np.float64)
                    assert np.all(np.abs(fw - fd) <= 1e-12), (label, r, q, i, fw, fd)  # weights in [0, 1]
                    gw, gd = w[PW_GAIN_G:].view(np.float64), d[PW_GAIN_G:].view(np.float64)
                    assert np.all(np.abs(gw - gd) <= 1e-13 * np.abs(gd)), (label, r, q, i, gw, gd)
                    checked += 1
        assert checked > 0, label


def _header_noise(hdr):
    """plan_key_noise from dense records' header words (tree_plan.h PW_HDR: flags, then the
    upstream dipole of glottis / tongue 1 / tongue 2 / lip)."""
    hdr = hdr.astype(np.uint64)
    m = np.zeros(hdr.shape, dtype=np.uint64)
    for c in range(4):
        on = ((hdr >> np.uint64(c)) & np.uint64(1)).astype(bool)
        up = ((hdr >> np.uint64(8 * (c + 1))) & np.uint64(0xFF)).astype(np.int64)
        dn = np.where(up < 39, up + 1, 40)
        bits = (np.uint64(1) << up.astype(np.uint64)) | (np.uint64(1) << dn.astype(np.uint64)) | \
            (np.uint64(1) << np.uint64(48 + c))
        m |= np.where(on, bits, np.uint64(0))
    return m


def test_hop_noise_mask_covers_every_sample(lib, oracle):
    """A hop record's noise mask (K1's choice of its noise phases' variant) is the union over the
    hop's samples of the dipoles their decisions target and the constrictions present, as the
    per-sample records' headers give them -- for decided and for mixed hops."""
    for label, frames, hop in _cases(oracle):
        rows, F = frames.shape
        n = (F - 1) * hop
        hops = np.zeros((rows, F - 1), dtype=HOP_DTYPE)
        assert lib.emu_plan_hops(frames.ctypes.data, rows, F, hop, 0, n, 44100.0, 0, hops.ctypes.data) == 0
        dense = np.zeros((rows, n, PLAN_WORDS), dtype=np.uint64)
        assert lib.emu_plan_records(frames.ctypes.data, rows, F, hop, 0, n, 44100.0, 0, dense.ctypes.data) == 0
        want = np.bitwise_or.reduce(_header_noise(dense[..., 0]).reshape(rows, F - 1, hop), axis=2)
        assert np.array_equal(hops["noise"], want), label
        assert (hops["noise"] >> np.uint64(48) & np.uint64(1)).all(), label  # the glottis source is always present
