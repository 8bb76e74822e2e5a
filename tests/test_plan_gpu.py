"""K5 (the noise-source plan kernel, csrc/tds_plan.hip) against the host restatement of the same
function (csrc/tree_plan.h plan_sample run on the CPU, tests/emu/plan_emu.cpp emu_plan_records),
record by record and word by word.

The plan holds everything calcNoiseSources decides from the geometry (TdsModel.cpp:1188-1508):
the constriction flags, the upstream sections of the dipole sources, the X_UN offsets of the
narrowest sections, the downstream factors, the area terms.  Every word is compared bit for bit
-- a flag or index that differs would move a noise source -- except the glottis dipole gain
0.5e-7 * 10^(dB / 20) (TdsModel.cpp:1546), whose pow comes from the device libm on the GPU and
from glibc on the host: it is held to 1 ulp.  Frames: config 2 (static vowels, hop 441: the
frames staged in LDS), config 5 (fricatives with the velum at 1.0 cm^2), config 3 (VCV target
sequences, one frame per sample: the global-memory path) and both glottis models."""
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
    lib_path = os.path.join(EMU, "libplan_emu.so")
    if not os.path.exists(lib_path):
        subprocess.check_call(["make", "-s", "-C", EMU])
    lib = ctypes.CDLL(lib_path)
    vp = ctypes.c_void_p
    lib.emu_plan_records.restype = ctypes.c_int
    lib.emu_plan_records.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long, ctypes.c_long,
                                     ctypes.c_double, ctypes.c_int, vp]

    def run(frames, hop, s0, s1, fs, two_mass):
        frames = np.ascontiguousarray(frames)
        rows, F = frames.shape
        out = np.zeros((rows, s1 - s0, PLAN_WORDS), dtype=np.uint64)
        rc = lib.emu_plan_records(frames.ctypes.data, rows, F, hop, s0, s1, fs, int(two_mass), out.ctypes.data)
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


@pytest.mark.parametrize("two_mass", (False, True))
def test_plan_records_config2_static_vowels(contexts, host_plans, two_mass):
    from areafunctionsynthesis_amd.workloads import build_frames, static_vowels
    ctx = contexts(44100.0, "tree", two_mass)
    w = static_vowels(24, seconds=1.0, fs=44100.0)
    frames = build_frames(w, ctx.af_to_frames)
    # a launch's range that starts mid-hop and one at the end of the utterance
    for s0, s1 in ((0, 4096), (12345, 12345 + 2000), ((frames.shape[1] - 1) * w.hop - 1500,
                                                        (frames.shape[1] - 1) * w.hop)):
        g = ctx.noise_plans(frames, w.hop, s0, s1)
        h = host_plans(frames, w.hop, s0, s1, 44100.0, two_mass)
        _compare(g, h, f"config 2 [two_mass={two_mass}] samples {s0}..{s1}")


@pytest.mark.parametrize("two_mass", (False, True))
def test_plan_records_config5_fricatives(contexts, host_plans, two_mass):
    from areafunctionsynthesis_amd.workloads import build_frames, fricatives
    ctx = contexts(44100.0, "tree", two_mass)
    w = fricatives(27, seconds=0.5, fs=44100.0, velum_cm2=1.0)
    frames = build_frames(w, ctx.af_to_frames)
    n = (frames.shape[1] - 1) * w.hop
    g = ctx.noise_plans(frames, w.hop, 0, n)
    h = host_plans(frames, w.hop, 0, n, 44100.0, two_mass)
    _compare(g, h, f"config 5 [two_mass={two_mass}]")
    # the fricatives do drive the tongue / lip sources: the comparison covers set flags
    flags = g[..., 0] & 0xFF
    assert np.count_nonzero(flags & 2) > 0 and np.count_nonzero(flags & 8) > 0


def test_plan_records_config3_vcv(contexts, host_plans, oracle):
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
    ctx = contexts(22050.0, "tree", False)
    n = frames.shape[1] - 1
    g = ctx.noise_plans(frames, 1, 0, n)
    h = host_plans(frames, 1, 0, n, 22050.0, False)
    _compare(g, h, "config 3")
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


# ---------------------------------------------------------------------------
# Hop mode (hops >= 32, the tree solver's default there): K5's hop records against the host
# reference plan_hop_host (tests/emu/plan_emu.cpp emu_plan_hops), and the dense records of the
# mixed hops' samples against plan_sample.
# ---------------------------------------------------------------------------
HOP_DTYPE = np.dtype([("p", "<u8", (PLAN_WORDS, 4)), ("kind", "u1", (PLAN_WORDS,)), ("mixed", "<u4"),
                      ("dense", "<u4"), ("noise", "<u8")])
assert HOP_DTYPE.itemsize == 544


@pytest.fixture(scope="module")
def host_hops():
    lib = ctypes.CDLL(os.path.join(EMU, "libplan_emu.so"))
    vp = ctypes.c_void_p
    lib.emu_plan_hops.restype = ctypes.c_int
    lib.emu_plan_hops.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long, ctypes.c_long,
                                  ctypes.c_double, ctypes.c_int, vp]

    def run(frames, hop, s0, s1, fs, two_mass):
        frames = np.ascontiguousarray(frames)
        rows, F = frames.shape
        slots = (s1 - 1) // hop - s0 // hop + 1
        out = np.zeros((rows, slots), dtype=HOP_DTYPE)
        assert lib.emu_plan_hops(frames.ctypes.data, rows, F, hop, s0, s1, fs, int(two_mass), out.ctypes.data) == 0
        return out
    return run


def _compare_hops(ctx, host_hops, host_plans, frames, hop, s0, s1, fs, two_mass, label):
    gh, gp = ctx.noise_plan_hops(frames, hop, s0, s1)
    gh = gh.view(HOP_DTYPE)[..., 0]
    hh = host_hops(frames, hop, s0, s1, fs, two_mass)
    assert np.array_equal(gh["mixed"], hh["mixed"]), label
    assert np.array_equal(gh["kind"], hh["kind"]), label
    assert np.array_equal(gh["noise"], hh["noise"]), label  # (the dipoles and constrictions of every sample)
    gw, hw = gh["p"].copy(), hh["p"].copy()
    # the glottis gain (a constant word: p[15][0]) comes from the device pow: 1 ulp
    ulps = np.abs(gw[..., 15, 0].view(np.int64) - hw[..., 15, 0].view(np.int64))
    assert ulps.max() <= 1, (label, int(ulps.max()))
    gw[..., 15, 0] = hw[..., 15, 0] = 0
    diff = gw != hw
    if diff.any():
        r, q, w, j = np.argwhere(diff)[0]
        raise AssertionError(f"{label}: {int(diff.sum())} inputs differ; first: row {r} slot {q} word {w} input {j}")
    # the mixed hops' samples: their dense records
    mixed_samples = np.zeros(gp.shape[:2], dtype=bool)
    for r, q in np.argwhere(gh["mixed"] != 0):
        h = s0 // hop + q
        lo, hi = max(h * hop, s0), min((h + 1) * hop, s1)
        mixed_samples[r, lo - s0:hi - s0] = True
    if mixed_samples.any():
        hp = host_plans(frames, hop, s0, s1, fs, two_mass)
        _compare(gp[mixed_samples][None], hp[mixed_samples][None], label + " (mixed hops' dense records)")
    assert not gp[~mixed_samples].any(), label  # nothing written for the other samples
    return int(np.count_nonzero(gh["mixed"])), gh.size


@pytest.mark.parametrize("two_mass", (False, True))
def test_plan_hops_config2_config5(contexts, host_hops, host_plans, two_mass):
    from areafunctionsynthesis_amd.workloads import build_frames, fricatives, static_vowels
    ctx = contexts(44100.0, "tree", two_mass)
    for w in (static_vowels(24, seconds=0.5, fs=44100.0), fricatives(27, seconds=0.5, fs=44100.0, velum_cm2=1.0)):
        frames = build_frames(w, ctx.af_to_frames)
        n = (frames.shape[1] - 1) * w.hop
        for s0, s1 in ((0, n), (12345, 12345 + 2000)):
            mixed, total = _compare_hops(ctx, host_hops, host_plans, frames, w.hop, s0, s1, 44100.0, two_mass,
                                         f"{w.name} two_mass={two_mass} samples {s0}..{s1}")
            assert mixed == 0, (w.name, mixed, total)  # static shapes: one decision per hop


def test_plan_hops_transitions(contexts, host_hops, host_plans, oracle):
    """Frame-rate VCV trajectories (hop 441: the constrictions form and release inside hops, so
    some hops are mixed) and transitions between all Default.params shapes."""
    from areafunctionsynthesis_amd.frames import DEFAULT_GLOTTIS
    from areafunctionsynthesis_amd.params import default_shapes
    from areafunctionsynthesis_amd.workloads import build_frames, vcv
    ctx = contexts(44100.0, "tree", False)
    w = vcv(16, fs=44100.0)
    frames = build_frames(w, ctx.af_to_frames)
    n = (frames.shape[1] - 1) * w.hop
    mixed, total = _compare_hops(ctx, host_hops, host_plans, frames, w.hop, 0, n, 44100.0, False, "vcv frames")
    sh = default_shapes()
    names = sorted(sh)
    frames = np.stack([np.stack([oracle.af_to_frame(sh[names[(k + j) % len(names)]]) for j in range(6)])
                       for k in range(len(names))]).astype(FRAME_DTYPE)
    frames["glottis"] = DEFAULT_GLOTTIS
    m2, t2 = _compare_hops(ctx, host_hops, host_plans, frames, 97, 0, 5 * 97, 44100.0, False, "all shapes")
    assert 0 < mixed + m2 < total + t2


def test_hop_words_vs_dense_records(contexts):
    """The plan words the synthesis kernel evaluates per sample from a hop record
    (plan_word_fast, compiled with K1's flags: afs_plan_hop_words) against K5's dense records of
    the same samples, word kind by word kind, on static vowels and fricatives (hop 441, every
    sample of the undecided-free hops).  The discrete words and sqrt(A) are bit-identical; the
    quotients 1/A and 1/sqrt(4A/pi) come from v_rcp_f64 + one Newton step + a residual correction
    (tree_core.h fast_div) instead of IEEE divisions and the downstream factors from hop-end values:
    their distance to the dense records is measured here (ulps / relative) and bounded."""
    from areafunctionsynthesis_amd.workloads import build_frames, fricatives, static_vowels
    ctx = contexts(44100.0, "tree", False)
    rng = np.random.default_rng(5)
    worst = {}
    for w in (static_vowels(8, seconds=0.05, fs=44100.0), fricatives(9, seconds=0.05, fs=44100.0, velum_cm2=1.0)):
        frames = build_frames(w, ctx.af_to_frames)
        n = (frames.shape[1] - 1) * w.hop
        hops, _ = ctx.noise_plan_hops(frames, w.hop, 0, n)
        dense = ctx.noise_plans(frames, w.hop, 0, n)
        rec = hops.view(HOP_DTYPE)[..., 0]
        rows, slots = rec.shape
        # every sample of 4 random hops per row (plus the first and last sample of every hop)
        pick, ratios = [], []
        for r in range(rows):
            for q in range(slots):
                if rec["mixed"][r, q]:
                    continue
                idx = np.unique(np.concatenate([[0, w.hop - 1], rng.integers(0, w.hop, 24)]))
                for i in idx:
                    pick.append((r, q, int(i)))
        hrec = np.stack([hops[r, q] for r, q, _ in pick])
        ratio = np.array([i / w.hop for _, _, i in pick])
        got = ctx.plan_hop_words(hrec, ratio)
        want = np.stack([dense[r, q * w.hop + i] for r, q, i in pick])
        kinds = np.stack([rec["kind"][r, q] for r, q, _ in pick])
        for k, name in ((0, "const"), (1, "1/A"), (2, "sqrtA"), (3, "1/d"), (4, "N/D")):
            m = kinds == k
            m[:, PW_GAIN_G] = False  # (the gain: hop-constant, checked below)
            if not m.any():
                continue
            g, h = got[m].view(np.int64), want[m].view(np.int64)
            if k in (0, 2):
                assert np.array_equal(g, h), (w.name, name, int(np.count_nonzero(g != h)))
                worst[name] = 0
                continue
            gf, hf = got[m].view(np.float64), want[m].view(np.float64)
            rel = np.abs(gf - hf) / np.abs(hf)
            ulps = np.abs(g - h)
            worst[name] = max(worst.get(name, 0), int(ulps.max()))
            bound = 1e-12 if k == 4 else 1e-14
            assert rel.max() <= bound, (w.name, name, float(rel.max()), int(ulps.max()))
        gain = got[:, PW_GAIN_G].view(np.float64)
        assert np.all(np.abs(gain - want[:, PW_GAIN_G].view(np.float64)) <= 1e-13 * np.abs(gain)), w.name
    print("hop words vs dense records, max ulps by kind:", worst)
    assert worst["1/A"] <= 16 and worst["1/d"] <= 16, worst
