"""CPU check of the cooperative tree kernel's decomposition (test-only host build of
csrc/tree_core.h, see tests/emu/tree_emu.cpp): lane ownership, LDS exchange and the
arm-solver LDL^T reproduce the oracle to rounding level, for any lane width."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from areafunctionsynthesis_amd.frames import FRAME_DTYPE

EMU = os.path.join(os.path.dirname(os.path.abspath(__file__)), "emu")
TOL = 1e-9


@pytest.fixture(scope="module")
def emu():
    subprocess.check_call(["make", "-s", "-C", EMU])
    lib = ctypes.CDLL(os.path.join(EMU, "libtree_emu.so"))
    vp = ctypes.c_void_p
    lib.emu_tree_utterance.restype = ctypes.c_long
    lib.emu_tree_utterance.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_double,
                                       ctypes.c_int, vp, vp, vp, ctypes.c_int]
    lib.emu_tree_rounds.restype = ctypes.c_int
    lib.emu_tree_rounds.argtypes = [ctypes.c_double]

    def run(fr, hop, seed, fs, W=16):
        fr = np.ascontiguousarray(fr, dtype=FRAME_DTYPE)
        out = np.zeros((fr.size - 1) * hop)
        dummy = np.zeros(97)
        n = lib.emu_tree_utterance(fr.ctypes.data, fr.size, hop, seed, fs, W, out.ctypes.data,
                                   dummy.ctypes.data, dummy.ctypes.data, 0)
        assert n == out.size
        return out
    lib.emu_tree_utterance_opt.restype = ctypes.c_long
    lib.emu_tree_utterance_opt.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_double, vp,
                                           ctypes.c_double, vp]

    def run_opt(fr, hop, seed, fs, opt):
        from oracle_lib import OPTION_DEFAULTS
        o = dict(OPTION_DEFAULTS, **opt)
        iopt = np.array([o[k] for k in ("turbulence_losses", "soft_walls", "generate_noise_sources",
                                        "radiation_from_skin", "piriform_fossa", "inner_length_corrections",
                                        "transvelar_coupling", "glottis_loss", "glottis_model")], dtype=np.int32)
        fr = np.ascontiguousarray(fr, dtype=FRAME_DTYPE)
        out = np.zeros((fr.size - 1) * hop)
        n = lib.emu_tree_utterance_opt(fr.ctypes.data, fr.size, hop, seed, fs, iopt.ctypes.data,
                                       float(o["flow_separation_area_ratio"]), out.ctypes.data)
        assert n == out.size
        return out
    run.lib = lib
    run.opt = run_opt
    return run


def test_schedule_is_valid(emu):
    # build_tables checks the arm partition (every current and every edge of the graph in
    # exactly one role) and reports -1 otherwise; else the arm reduction's 6 sequential steps
    assert emu.lib.emu_tree_rounds(22050.0) == 6  # afs_tables.cpp arm_records


def test_golden_utterances(emu, golden_dir):
    g = np.load(os.path.join(golden_dir, "utterances.npz"), allow_pickle=False)
    frames = g["frames"].view(FRAME_DTYPE)
    n = g["out"].shape[1]
    for i, name in enumerate(g["names"]):
        fr = frames[i, : g["num_frames"][i]]
        y = emu(fr, int(g["hop"][i]), int(g["seed"][i]), float(g["fs"][i]))[:n]
        assert np.abs(y - g["out"][i]).max() <= TOL, name


@pytest.mark.parametrize("W", [32, 64])
def test_lane_width_invariance(emu, golden_dir, W):
    """The decomposition does not change the arithmetic: any lane width gives bitwise
    the same audio as W = 16."""
    g = np.load(os.path.join(golden_dir, "utterances.npz"), allow_pickle=False)
    frames = g["frames"].view(FRAME_DTYPE)
    for i in (0, 3, 6):
        fr = frames[i, : g["num_frames"][i]]
        args = (int(g["hop"][i]), int(g["seed"][i]), float(g["fs"][i]))
        assert np.array_equal(emu(fr, *args, W=W), emu(fr, *args, W=16))


@pytest.mark.parametrize("opt", [{"transvelar_coupling": 1}, {"glottis_loss": 1}, {"glottis_loss": 2},
                                 {"flow_separation_area_ratio": 1.2}, {"piriform_fossa": 1, "soft_walls": 0},
                                 {"transvelar_coupling": 1, "glottis_loss": 2, "generate_noise_sources": 0},
                                 {"glottis_model": 1}],
                         ids=lambda o: "+".join(f"{k}={v}" for k, v in o.items()))
def test_options_vs_oracle(emu, oracle, opt):
    """The tree decomposition of every TdsModel option (the SOR solver runs in the lane kernel)."""
    from areafunctionsynthesis_amd.frames import DEFAULT_GLOTTIS
    from areafunctionsynthesis_amd.params import default_shapes
    sh = default_shapes()
    f = oracle.af_to_frame(sh["a:"])
    f["velum_opening_cm2"] = 0.5
    f["glottis"] = DEFAULT_GLOTTIS
    g = oracle.af_to_frame(sh["z"])
    g["velum_opening_cm2"] = 0.5
    g["glottis"] = [110.0, 8000.0, 0.02, 0.01, 0.0, -30.0]
    if opt.get("glottis_model"):  # control 5 is the two-mass model's damping factor
        f["glottis"][5], g["glottis"][5] = 1.0, 1.5
    frames = np.stack([f, g, g, f])
    for fs, hop in ((22050.0, 300), (44100.0, 441)):
        x = emu.opt(frames, hop, 5, fs, opt)
        y = oracle.utterance(frames, hop, 5, fs, opt=opt)
        assert np.abs(x[:2048] - y[:2048]).max() <= TOL, fs
        assert np.sqrt(np.mean((x - y) ** 2)) < 1e-8, fs


@pytest.mark.parametrize("hop", [7, 31, 32, 97])
def test_output_stage_paths_vs_oracle(emu, oracle, hop):
    """Hops below OUT_DEFER_MIN_HOP (32) run the output filter inside the sample step, longer
    hops once per hop over the hop's flows (tree_core.h output_filter_run); both match the
    oracle, including across frame transitions."""
    from areafunctionsynthesis_amd.frames import DEFAULT_GLOTTIS
    from areafunctionsynthesis_amd.params import default_shapes
    sh = default_shapes()
    frames = []
    for name, f0 in (("a:", 120.0), ("i:", 130.0), ("s", 125.0), ("u:", 110.0), ("a:", 118.0)):
        f = oracle.af_to_frame(sh[name])
        f["glottis"] = DEFAULT_GLOTTIS
        f["glottis"][0] = f0
        frames.append(f)
    frames = np.stack(frames * 6)
    x = emu.opt(frames, hop, 3, 22050.0, {})
    y = oracle.utterance(frames, hop, 3, 22050.0)
    assert x.size == y.size == (frames.size - 1) * hop
    assert np.abs(x - y).max() <= TOL


def test_noise_plan_every_shape_vs_oracle(emu, oracle):
    """The noise-source plan (tree_plan.h: the constriction scans ahead of the time loop) on
    every shape of Default.params, through transitions between shapes that move constrictions
    in and out of the tongue / lip / teeth cases, with velum and laterality: the emulator
    (plan + synthesis step) against the oracle's in-loop scans (TdsModel.cpp:1188-1604)."""
    from areafunctionsynthesis_amd.frames import DEFAULT_GLOTTIS
    from areafunctionsynthesis_amd.params import default_shapes
    sh = default_shapes()
    names = sorted(sh)
    rng = np.random.default_rng(11)
    hop, fs = 53, 44100.0
    for k in range(0, len(names), 3):
        seq = [names[(k + j) % len(names)] for j in range(4)]
        frames = np.stack([oracle.af_to_frame(sh[n]) for n in seq])
        frames["glottis"] = DEFAULT_GLOTTIS
        frames["glottis"][:, 5] = -30.0 + 10.0 * rng.random(4)
        frames["velum_opening_cm2"] = rng.random(4) * (k % 2)
        frames["laterality"][:, 30:36] = 0.2 * rng.random((4, 6)) * (k % 3 == 0)
        x = emu(frames, hop, k + 1, fs)
        y = oracle.utterance(frames, hop, k + 1, fs)
        assert np.abs(x - y).max() <= TOL, seq


@pytest.fixture
def hop_mode(emu):
    """The emulator with hop records (tree_plan.h PlanHop) at hops >= PLAN_HOP_MIN (32)."""
    lib = emu.lib
    lib.emu_tree_set_hop_mode.argtypes = [ctypes.c_int]
    lib.emu_tree_hop_counts.argtypes = [ctypes.c_void_p, ctypes.c_void_p]

    def counts():
        h, m = ctypes.c_long(), ctypes.c_long()
        lib.emu_tree_hop_counts(ctypes.byref(h), ctypes.byref(m))
        return h.value, m.value
    lib.emu_tree_set_hop_mode(1)
    counts()
    yield counts
    lib.emu_tree_set_hop_mode(0)


def test_hop_mode_golden_utterances(emu, golden_dir, hop_mode):
    """Hop records instead of per-sample records: the plan words of a hop whose samples share
    the plan's decisions are evaluated from the hop's inputs at every sample (area terms bit for
    bit, downstream factors within ulps); the goldens hold at the same tolerance."""
    g = np.load(os.path.join(golden_dir, "utterances.npz"), allow_pickle=False)
    frames = g["frames"].view(FRAME_DTYPE)
    n = g["out"].shape[1]
    for i, name in enumerate(g["names"]):
        fr = frames[i, : g["num_frames"][i]]
        hop = int(g["hop"][i])
        y = emu(fr, hop, int(g["seed"][i]), float(g["fs"][i]))[:n]
        assert np.abs(y - g["out"][i]).max() <= TOL, name
    hops, mixed = hop_mode()
    assert hops > 0 and mixed < hops


def test_hop_mode_every_shape_vs_oracle(emu, oracle, hop_mode):
    """Hop mode through transitions between all shapes of Default.params (constrictions moving in
    and out of the tongue / lip / teeth cases within a hop: mixed hops take the dense records),
    with the aspiration strength constant per utterance (the hop records' glottis gain)."""
    from areafunctionsynthesis_amd.frames import DEFAULT_GLOTTIS
    from areafunctionsynthesis_amd.params import default_shapes
    sh = default_shapes()
    names = sorted(sh)
    rng = np.random.default_rng(12)
    hop, fs = 97, 44100.0
    for k in range(0, len(names), 3):
        seq = [names[(k + j) % len(names)] for j in range(4)]
        frames = np.stack([oracle.af_to_frame(sh[n]) for n in seq] + [oracle.af_to_frame(sh[seq[-1]])])
        frames["glottis"] = DEFAULT_GLOTTIS
        frames["glottis"][:, 5] = -30.0 + 10.0 * rng.random()
        frames["velum_opening_cm2"] = rng.random(5) * (k % 2)
        frames["laterality"][:, 30:36] = 0.2 * rng.random((5, 6)) * (k % 3 == 0)
        x = emu(frames, hop, k + 1, fs)
        y = oracle.utterance(frames, hop, k + 1, fs)
        assert np.abs(x - y).max() <= TOL, seq
    hops, mixed = hop_mode()
    assert 0 < mixed < hops, (hops, mixed)


@pytest.mark.parametrize("hop", [7, 97, 441])
@pytest.mark.parametrize("skin", [1, 0])
def test_tone_in_k6_vs_in_step(emu, oracle, hop, skin):
    """The device default leaves the glottal-tone (skin radiation) filter out of the sample step:
    the synthesis kernel stores section 25's new pressure (lane 2, slot 0) per sample and K6 runs
    the filter in the output filter's loop (tree_core.h tone_output_run, TdsModel.cpp:687-705).
    Emulated that way, deferred hops give bitwise the audio of the in-step filter, and every hop
    length matches the oracle."""
    from areafunctionsynthesis_amd.frames import DEFAULT_GLOTTIS
    from areafunctionsynthesis_amd.params import default_shapes
    lib = emu.lib
    lib.emu_tree_set_tone_k6.argtypes = [ctypes.c_int]
    sh = default_shapes()
    frames = []
    for name, f0 in (("a:", 120.0), ("s", 125.0), ("i:", 130.0)):
        f = oracle.af_to_frame(sh[name])
        f["glottis"] = DEFAULT_GLOTTIS
        f["glottis"][0] = f0
        frames.append(f)
    frames = np.stack(frames * 3)
    opt = {"radiation_from_skin": skin}
    lib.emu_tree_set_tone_k6(1)
    try:
        x = emu.opt(frames, hop, 7, 22050.0, opt)
    finally:
        lib.emu_tree_set_tone_k6(0)
    y = emu.opt(frames, hop, 7, 22050.0, opt)
    if hop >= 32:  # OUT_DEFER_MIN_HOP: both defer the output filter
        assert np.array_equal(x, y)
    z = oracle.utterance(frames, hop, 7, 22050.0, opt=opt)
    assert np.abs(x - z).max() <= TOL


@pytest.mark.parametrize("W", [16, 64])
def test_noise_variants_bitwise(emu, oracle, hop_mode, W):
    """The noise-phase variants (tree_core.h NoiseV: the glottis source alone, glottis + first
    tongue constriction below dipole 32, ...) chosen per hop from the hop record's noise mask and
    the slots still holding amplitude, as the device chooses them per launch: the audio is the
    full phases' bit for bit -- vowels (light variants), fricatives, and transitions between all
    shapes (constrictions appearing and dying away across hops, a decaying amplitude keeping its
    slot in the heavier variant)."""
    from areafunctionsynthesis_amd.frames import DEFAULT_GLOTTIS
    from areafunctionsynthesis_amd.params import default_shapes
    lib = emu.lib
    lib.emu_tree_set_noise_variants.argtypes = [ctypes.c_int]
    lib.emu_tree_variant_counts.argtypes = [ctypes.c_void_p]
    sh = default_shapes()
    names = sorted(sh)
    rng = np.random.default_rng(21)
    cases = []
    for seq in (["a:"] * 4, ["i:"] * 4, ["s"] * 4, ["u:", "S", "a:", "f"], ["(a)b(a):", "i:", "l", "u:"]):
        cases.append(seq)
    for k in range(0, len(names), 5):
        cases.append([names[(k + j) % len(names)] for j in range(4)])
    used = np.zeros(4, dtype=np.int64)
    for n, seq in enumerate(cases):
        frames = np.stack([oracle.af_to_frame(sh[x]) for x in seq] + [oracle.af_to_frame(sh[seq[-1]])])
        frames["glottis"] = DEFAULT_GLOTTIS
        frames["glottis"][:, 0] = 100.0 + 10.0 * rng.random(5)
        frames["velum_opening_cm2"] = rng.random(5) * (n % 2)
        ys = []
        for on in (0, 1):
            lib.emu_tree_set_noise_variants(on)
            try:
                ys.append(emu(frames, 97, n + 1, 44100.0, W=W))
            finally:
                lib.emu_tree_set_noise_variants(0)
            c = np.zeros(4, dtype=np.int64)
            lib.emu_tree_variant_counts(c.ctypes.data)
            used += c
        assert np.array_equal(ys[0], ys[1]), (seq, W)
    assert used[0] > 0 and used[3] > 0, used  # (the full phases and the glottis-only variant both ran)
    if W == 16:
        assert used[1] > 0 and used[2] > 0, used  # (and both tongue variants)
    hop_mode()


@pytest.mark.parametrize("case", ["tiny_pharynx", "alternating", "wide_open"])
def test_arm_scan_extreme_areas_vs_oracle(emu, oracle, case):
    """The arm solver's lane scans (tree_core.h solve_arms, AFS_ARM_SCAN) on tracts far outside
    speech: sections at the area clamp beside 60 cm^2 sections, a whole pharynx at the clamp, every
    section wide open.  The pivot recurrence's 2 x 2 products span up to 8 lanes, an arm's first lane
    included (its F = 0 makes the ratio, not the magnitude, independent of the lanes before it): the
    products of up to 8 pivots must stay inside the fp64 range for any tract the model accepts (the
    diagonal is bounded by the area clamp, ~1e7 at 44.1 kHz).  The emulator's audio stays finite and
    equals the oracle's sequential Cholesky to the usual tolerance, relative to the signal."""
    from areafunctionsynthesis_amd.frames import DEFAULT_GLOTTIS
    from areafunctionsynthesis_amd.params import default_shapes
    f = oracle.af_to_frame(default_shapes()["a:"])
    f["glottis"] = DEFAULT_GLOTTIS
    f["velum_opening_cm2"] = 2.0
    a = f["area_cm2"]
    if case == "tiny_pharynx":
        a[:20] = 0.0011
    elif case == "alternating":
        a[:] = np.where(np.arange(a.size) % 2 == 0, 0.0011, 60.0)
    else:
        a[:] = 60.0
    f["area_cm2"] = a
    frames = np.stack([f] * 6)
    for fs, hop in ((22050.0, 256), (44100.0, 441)):
        x = emu(frames, hop, 3, fs)
        y = oracle.utterance(frames, hop, 3, fs)
        assert np.all(np.isfinite(x)) and np.all(np.isfinite(y)), (case, fs)
        scale = max(1.0, float(np.abs(y).max()))
        assert np.abs(x[:2048] - y[:2048]).max() <= TOL * scale, (case, fs)


@pytest.fixture(scope="module")
def pair_emu():
    subprocess.check_call(["make", "-s", "-C", EMU])
    lib = ctypes.CDLL(os.path.join(EMU, "libpair_emu.so"))
    vp = ctypes.c_void_p
    lib.emu_pair_utterance.restype = ctypes.c_long
    lib.emu_pair_utterance.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_double, ctypes.c_int,
                                       vp, ctypes.c_double, vp, vp]
    return lib


@pytest.mark.parametrize("W", [16, 64])
@pytest.mark.parametrize("opt", [{}, {"glottis_model": 1}, {"glottis_loss": 2, "transvelar_coupling": 1},
                                 {"radiation_from_skin": 0, "generate_noise_sources": 0}],
                         ids=lambda o: "+".join(f"{k}={v}" for k, v in o.items()) or "default")
def test_wave_pair_step_equals_one_wave(emu, pair_emu, oracle, W, opt):
    """The wave pairs (tree_core.h sample_step_pair, the device's throughput and voice kernels): the
    DYN and STAT roles on two threads meeting at the step's barriers (tests/emu/pair_emu.cpp) give
    the one-wave step's audio (tone filter in K6, as on the device) and rand() count bit for bit --
    the lean solver, the glottis committed by STAT, the rand() blocks generated on DYN included."""
    from oracle_lib import OPTION_DEFAULTS

    from areafunctionsynthesis_amd.frames import DEFAULT_GLOTTIS
    from areafunctionsynthesis_amd.params import default_shapes
    if W == 64 and opt:
        pytest.skip("the one-wave emulator takes options at 16 lanes (lane-width invariance: test_lane_width_invariance)")
    sh = default_shapes()
    frames = []
    for name, f0, velum in (("a:", 120.0, 0.0), ("s", 125.0, 0.3), ("i:", 130.0, 0.0), ("z", 118.0, 0.5)):
        f = oracle.af_to_frame(sh[name])
        f["glottis"] = DEFAULT_GLOTTIS
        f["glottis"][0] = f0
        f["velum_opening_cm2"] = velum
        if opt.get("glottis_model"):
            f["glottis"][5] = 1.2
        frames.append(f)
    frames = np.ascontiguousarray(np.stack(frames * 2), dtype=FRAME_DTYPE)
    hop, fs, seed = 300, 22050.0, 11
    o = dict(OPTION_DEFAULTS, **opt)
    iopt = np.array([o[k] for k in ("turbulence_losses", "soft_walls", "generate_noise_sources", "radiation_from_skin",
                                    "piriform_fossa", "inner_length_corrections", "transvelar_coupling",
                                    "glottis_loss", "glottis_model")], dtype=np.int32)
    y = np.zeros((frames.size - 1) * hop)
    draws = np.zeros(1, np.uint64)
    n = pair_emu.emu_pair_utterance(frames.ctypes.data, frames.size, hop, seed, fs, W, iopt.ctypes.data,
                                    float(o["flow_separation_area_ratio"]), y.ctypes.data, draws.ctypes.data)
    assert n == y.size
    emu.lib.emu_tree_set_tone_k6.argtypes = [ctypes.c_int]
    emu.lib.emu_tree_set_tone_k6(1)
    try:
        x = emu.opt(frames, hop, seed, fs, opt) if W == 16 else emu(frames, hop, seed, fs, W=W)
    finally:
        emu.lib.emu_tree_set_tone_k6(0)
    assert np.isfinite(y).all()
    assert np.array_equal(x, y), np.abs(x - y).max()
    z = oracle.utterance(frames, hop, seed, fs, opt=opt)
    assert np.abs(y[:2048] - z[:2048]).max() <= TOL
    if o["generate_noise_sources"]:
        assert int(draws[0]) > 0
