"""CPU check of the segment-aligned kernel's decomposition (test-only host build of
csrc/seg_core.h, tests/emu/seg_emu.cpp): the lane partition, the static condensation (the
constant LDL^T of the trachea / nose / fossa subtrees and its lane scans), the dynamic walks,
arm reductions and the junction lane reproduce the reference to rounding level."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from areafunctionsynthesis_amd.frames import FRAME_DTYPE

EMU = os.path.join(os.path.dirname(os.path.abspath(__file__)), "emu")
TOL = 1e-9
OPT_KEYS = ("turbulence_losses", "soft_walls", "generate_noise_sources", "radiation_from_skin", "piriform_fossa",
            "inner_length_corrections", "transvelar_coupling", "glottis_loss", "glottis_model")


@pytest.fixture(scope="module")
def emu():
    subprocess.check_call(["make", "-s", "-C", EMU])
    lib = ctypes.CDLL(os.path.join(EMU, "libseg_emu.so"))
    vp = ctypes.c_void_p
    lib.emu_seg_utterance.restype = ctypes.c_long
    lib.emu_seg_utterance.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_double, vp,
                                      ctypes.c_double, vp, vp]
    lib.emu_seg_tables_ok.restype = ctypes.c_int
    lib.emu_seg_tables_ok.argtypes = [ctypes.c_double]

    def run(fr, hop, seed, fs, opt=None, draws=False):
        fr = np.ascontiguousarray(fr, dtype=FRAME_DTYPE)
        out = np.zeros((fr.size - 1) * hop)
        d = np.zeros(1, dtype=np.int64)
        iopt, ratio = None, 1.0
        if opt is not None:
            from oracle_lib import OPTION_DEFAULTS
            o = dict(OPTION_DEFAULTS, **opt)
            iopt = np.array([o[k] for k in OPT_KEYS], dtype=np.int32)
            ratio = float(o["flow_separation_area_ratio"])
        n = lib.emu_seg_utterance(fr.ctypes.data, fr.size, hop, seed, fs,
                                  iopt.ctypes.data if iopt is not None else None, ratio, out.ctypes.data, d.ctypes.data)
        assert n == out.size
        return (out, int(d[0])) if draws else out
    run.lib = lib
    return run


def test_partition_checks(emu):
    # build_seg_tables: every current in exactly one slot, every edge of the current graph in
    # exactly one role, the static LDL^T free of fill outside the chains, the kernel's fixed
    # lane roles (seg_tables.cpp)
    assert emu.lib.emu_seg_tables_ok(22050.0) == 1
    assert emu.lib.emu_seg_tables_ok(44100.0) == 1


def test_golden_utterances(emu, golden_dir):
    g = np.load(os.path.join(golden_dir, "utterances.npz"), allow_pickle=False)
    frames = g["frames"].view(FRAME_DTYPE)
    n = g["out"].shape[1]
    for i, name in enumerate(g["names"]):
        fr = frames[i, : g["num_frames"][i]]
        y = emu(fr, int(g["hop"][i]), int(g["seed"][i]), float(g["fs"][i]))[:n]
        assert np.abs(y - g["out"][i]).max() <= TOL, name


@pytest.mark.parametrize("opt", [{}, {"transvelar_coupling": 1}, {"glottis_loss": 1}, {"glottis_loss": 2},
                                 {"flow_separation_area_ratio": 1.2}, {"piriform_fossa": 1, "soft_walls": 0},
                                 {"turbulence_losses": 0, "inner_length_corrections": 0, "radiation_from_skin": 0},
                                 {"transvelar_coupling": 1, "glottis_loss": 2, "generate_noise_sources": 0},
                                 {"glottis_model": 1}],
                         ids=lambda o: "+".join(f"{k}={v}" for k, v in o.items()) or "defaults")
def test_options_vs_oracle(emu, oracle, opt):
    """Every TdsModel option through the seg decomposition."""
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
        x = emu(frames, hop, 5, fs, opt=opt)
        y = oracle.utterance(frames, hop, 5, fs, opt=opt)
        assert np.abs(x[:2048] - y[:2048]).max() <= TOL, fs
        assert np.sqrt(np.mean((x - y) ** 2)) < 1e-8, fs


@pytest.mark.parametrize("hop", [7, 31, 32, 97])
def test_output_stage_paths_vs_oracle(emu, oracle, hop):
    """Short hops filter inside the sample step, long hops once per hop (seg_output_filter_run)."""
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
    x = emu(frames, hop, 3, 22050.0)
    y = oracle.utterance(frames, hop, 3, 22050.0)
    assert x.size == y.size == (frames.size - 1) * hop
    assert np.abs(x - y).max() <= TOL


def test_noise_plan_every_shape_vs_oracle(emu, oracle):
    """Every shape of Default.params through transitions that move constrictions (tongue, lip,
    teeth cases), with velum and laterality; the rand() call count equals the oracle's."""
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
        x, draws = emu(frames, hop, k + 1, fs, draws=True)
        y = oracle.utterance(frames, hop, k + 1, fs)
        assert np.abs(x - y).max() <= TOL, seq
