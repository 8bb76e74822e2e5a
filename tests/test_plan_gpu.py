"""K5 (the noise-source plan kernel, csrc/tds_plan.hip) against the host restatement of the same
function (csrc/tree_plan.h plan_sample run on the CPU, tests/emu/seg_emu.cpp emu_plan_records),
record by record and word by word.

The plan holds everything calcNoiseSources decides from the geometry (TdsModel.cpp:1188-1508):
the constriction flags, the upstream sections of the dipole sources, the X_UN offsets of the
narrowest sections, the downstream factors, the area terms.  Every word is compared bit for bit
-- a flag or index that differs would move a noise source -- except the glottis dipole gain
0.5e-7 * 10^(dB / 20) (TdsModel.cpp:1546), whose pow comes from the device libm on the GPU and
from glibc on the host: it is held to 1 ulp.  Frames: config 2 (static vowels, hop 441: the
frames staged in LDS), config 5 (fricatives with the velum at 1.0 cm^2), config 3 (VCV target
sequences, one frame per sample: the global-memory path), both glottis models and both the tree
and the seg kernel's LDS offsets."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from areafunctionsynthesis_amd.frames import FRAME_DTYPE

pytestmark = pytest.mark.gpu

EMU = os.path.join(os.path.dirname(os.path.abspath(__file__)), "emu")
PW_GAIN_G = 15
PLAN_WORDS = 16


@pytest.fixture(scope="module")
def host_plans():
    lib_path = os.path.join(EMU, "libseg_emu.so")
    if not os.path.exists(lib_path):
        subprocess.check_call(["make", "-s", "-C", EMU])
    lib = ctypes.CDLL(lib_path)
    vp = ctypes.c_void_p
    lib.emu_plan_records.restype = ctypes.c_int
    lib.emu_plan_records.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long, ctypes.c_long,
                                     ctypes.c_double, ctypes.c_int, ctypes.c_int, vp]

    def run(frames, hop, s0, s1, fs, two_mass, seg):
        frames = np.ascontiguousarray(frames)
        rows, F = frames.shape
        out = np.zeros((rows, s1 - s0, PLAN_WORDS), dtype=np.uint64)
        rc = lib.emu_plan_records(frames.ctypes.data, rows, F, hop, s0, s1, fs, int(two_mass), int(seg),
                                  out.ctypes.data)
        assert rc == 0
        return out
    return run


@pytest.fixture(scope="module")
def contexts():
    from areafunctionsynthesis_amd.synthesizer import Context
    cache = {}

    def get(fs, solver, two_mass):
        key = (fs, solver, two_mass)
        if key not in cache:
            cache[key] = Context(fs, solver=solver, glottis_model=1 if two_mass else 0)
        return cache[key]
    yield get
    for c in cache.values():
        c.close()


def _compare(gpu, host, label):
    assert gpu.shape == host.shape
    exact = np.ones(PLAN_WORDS, dtype=bool)
    exact[PW_GAIN_G] = False
    diff = gpu[..., exact] != host[..., exact]
    if diff.any():
        r, t, w = np.argwhere(diff)[0]
        words = np.flatnonzero(exact)
        raise AssertionError(f"{label}: {int(diff.sum())} words differ; first: row {r} sample {t} word "
                             f"{words[w]}: gpu {int(gpu[r, t, words[w]]):#x} host {int(host[r, t, words[w]]):#x}")
    g = gpu[..., PW_GAIN_G].view(np.int64)
    h = host[..., PW_GAIN_G].view(np.int64)
    ulps = np.abs(g - h)  # (positive doubles: the bit patterns are ordered)
    assert ulps.max() <= 1, (label, int(ulps.max()))
    return int(np.count_nonzero(ulps))


def _cases():
    for solver in ("tree", "seg"):
        for two_mass in (False, True):
            yield solver, two_mass


@pytest.mark.parametrize("solver,two_mass", list(_cases()))
def test_plan_records_config2_static_vowels(contexts, host_plans, solver, two_mass):
    from areafunctionsynthesis_amd.workloads import build_frames, static_vowels
    ctx = contexts(44100.0, solver, two_mass)
    w = static_vowels(24, seconds=1.0, fs=44100.0)
    frames = build_frames(w, ctx.af_to_frames)
    # a launch's range that starts mid-hop and one at the end of the utterance
    for s0, s1 in ((0, 4096), (12345, 12345 + 2000), ((frames.shape[1] - 1) * w.hop - 1500,
                                                        (frames.shape[1] - 1) * w.hop)):
        g = ctx.noise_plans(frames, w.hop, s0, s1)
        h = host_plans(frames, w.hop, s0, s1, 44100.0, two_mass, solver == "seg")
        _compare(g, h, f"config 2 [{solver}, two_mass={two_mass}] samples {s0}..{s1}")


@pytest.mark.parametrize("solver,two_mass", list(_cases()))
def test_plan_records_config5_fricatives(contexts, host_plans, solver, two_mass):
    from areafunctionsynthesis_amd.workloads import build_frames, fricatives
    ctx = contexts(44100.0, solver, two_mass)
    w = fricatives(27, seconds=0.5, fs=44100.0, velum_cm2=1.0)
    frames = build_frames(w, ctx.af_to_frames)
    n = (frames.shape[1] - 1) * w.hop
    g = ctx.noise_plans(frames, w.hop, 0, n)
    h = host_plans(frames, w.hop, 0, n, 44100.0, two_mass, solver == "seg")
    _compare(g, h, f"config 5 [{solver}, two_mass={two_mass}]")
    # the fricatives do drive the tongue / lip sources: the comparison covers set flags
    flags = g[..., 0] & 0xFF
    assert np.count_nonzero(flags & 2) > 0 and np.count_nonzero(flags & 8) > 0


@pytest.mark.parametrize("solver", ("tree", "seg"))
def test_plan_records_config3_vcv(contexts, host_plans, oracle, solver):
    """Config 3 trajectories (the oracle's playTargetSequence frames, one per sample), the
    15 VCV sequences over their full length at 22.05 kHz."""
    from areafunctionsynthesis_amd.params import default_shapes
    sh = default_shapes()
    rows = []
    for v in ("a:", "e:", "i:", "o:", "u:"):
        for c in ("b", "d", "g"):
            s4 = np.stack([sh[v], sh[f"({v[0]}){c}({v[0]}):"], sh[v], sh[v]])
            rows.append(oracle.target_frames(s4, 22050.0))
    frames = np.stack(rows).astype(FRAME_DTYPE)
    ctx = contexts(22050.0, solver, False)
    n = frames.shape[1] - 1
    g = ctx.noise_plans(frames, 1, 0, n)
    h = host_plans(frames, 1, 0, n, 22050.0, False, solver == "seg")
    _compare(g, h, f"config 3 [{solver}]")
    flags = g[..., 0] & 0xFF
    assert np.count_nonzero(flags & 2) > 0  # the consonant closures form tongue constrictions


def test_plan_unsupported_solver():
    from areafunctionsynthesis_amd._native import AfsError
    from areafunctionsynthesis_amd.synthesizer import Context
    ctx = Context(22050.0, solver="cholesky")
    f = np.zeros((1, 3), dtype=FRAME_DTYPE)
    with pytest.raises(AfsError):
        ctx.noise_plans(f, 10)


def test_k1_interpolation_equals_k5_geometry(oracle):
    """The synthesis kernel's tube interpolation (frame_load + phase_interpolate, compiled in
    tds_tree.hip with the kernel's -ffp-contract=fast-honor-pragmas) is bit-identical to the uncontracted
    r1 * a + ratio * b that K5 (tree_plan.h PlanGeom), the host restatement and the reference
    (Tube::interpolate, Tube.cpp:438-505) evaluate: the constriction decisions K5 makes are made
    on the areas the tube network uses."""
    from areafunctionsynthesis_amd.params import default_shapes
    from areafunctionsynthesis_amd.synthesizer import Context
    sh = default_shapes()
    rng = np.random.default_rng(7)
    names = sorted(sh)
    n = 4096
    left = np.stack([oracle.af_to_frame(sh[names[k]]) for k in rng.integers(0, len(names), n)])
    right = np.stack([oracle.af_to_frame(sh[names[k]]) for k in rng.integers(0, len(names), n)])
    # areas below MIN_AREA on both sides (the clamps), and the ratios of every hop used
    left["area_cm2"][::7, 5] = 1e-5
    right["area_cm2"][::5, 6] = -0.3
    ratio = np.concatenate([np.arange(441) / 441.0, rng.random(n - 441)])
    ctx = Context(22050.0, solver="tree")
    area, length = ctx.tube_interpolate(left, right, ratio)
    amin = 0.001
    aL = np.maximum(left["area_cm2"], amin)
    aR = np.maximum(right["area_cm2"], amin)
    r1 = (1.0 - ratio)[:, None]
    r = ratio[:, None]
    a_ref = r1 * aL + r * aR  # numpy rounds each product: no fma
    a_ref = np.where(a_ref < amin, amin, a_ref)
    l_ref = r1 * left["length_cm"] + r * right["length_cm"]
    assert np.array_equal(area, a_ref), int(np.count_nonzero(area != a_ref))
    assert np.array_equal(length, l_ref), int(np.count_nonzero(length != l_ref))
    # (the check has teeth: a contracted fma(r1, a, ratio * b) -- evaluated here in extended
    # precision -- rounds differently for a share of these inputs)
    ld = np.longdouble
    a_fma = (ld(1.0) * r1.astype(ld) * aL.astype(ld) + (r * aR).astype(ld)).astype(np.float64)
    assert np.count_nonzero(a_fma != r1 * aL + r * aR) > 0
