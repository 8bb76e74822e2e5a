"""Synthesizer::playTargetSequence (Synthesizer.cpp:1286-1422).

The trajectory (interpolateParameters, F0 contour, lung-pressure fade-in / hold / fade-out,
area function -> tube per sample) lives in Synthesizer.cpp, which is not buildable here
(wxWidgets / portaudio), so it is pinned two ways:
* the C restatement (oracle ao_target_frames) against an independent pure-Python
  restatement that replays the reference's statements sample by sample, carrying
  glottisParams[PRESSURE] as state the way the reference does (bit-exact);
* the synthesis of those frames (one synthesizeSignalTds(tube_i, glottis_i, 1) per sample)
  against the reference build itself (oracle/_ref), bit-exact, and the committed
  tests/golden/target_seq.npz made from it for the GPU box.
GPU: afs_play_target_sequences against the golden vectors and the oracle, tolerance as
test_gpu_parity (1e-9 over the first 2048 samples, RMS < 1e-4 over the utterance)."""
import math
import os

import numpy as np
import pytest

from areafunctionsynthesis_amd.params import default_shapes

SHORT = {"stationary_s": [0.02, 0.01, 0.02, 0.01], "transition_s": [0.01, 0.01, 0.01]}
F0 = (100.0, 115.0, 105.0, 80.0)


def _python_trajectory(shapes4, fs, st, tr, P=8000.0):
    """The loop body of playTargetSequence (:1329-1420), statement by statement."""
    b = [st[0]]
    b.append(st[0] + tr[0])
    b.append(st[0] + tr[0] + st[1])
    b.append(st[0] + tr[0] + st[1] + tr[1])
    b.append(st[0] + tr[0] + st[1] + tr[1] + st[2])
    b.append(st[0] + tr[0] + st[1] + tr[1] + st[2] + tr[2])
    b.append(st[0] + tr[0] + st[1] + tr[1] + st[2] + tr[2] + st[3])
    total = b[6]
    n = int(fs * total)
    pressure = P  # sensorDataToGlottisParams
    f0s, prs, params = [], [], []
    cur = np.array(shapes4[0], dtype=np.float64)

    def interp(p0, p1, t0, t1, tx):
        return np.array([(p1[k] - p0[k]) / 2 * math.cos((t1 - tx) / (t1 - t0) * math.pi) + (p1[k] + p0[k]) / 2
                         for k in range(16)])

    for i in range(n):
        if i < 0.1 * fs:
            if i < 0.05 * fs:
                pressure = 0.0
            else:
                pressure = P / 2 * math.cos((0.1 * fs - i) / (0.05 * fs) * math.pi) + P / 2
        if i < b[1] * fs:
            f0 = (F0[0] + F0[1]) / 2 + (F0[1] - F0[0]) / 2 * math.cos((b[1] * fs - i) / (b[1] * fs) * math.pi)
        elif i < b[3] * fs:
            f0 = (F0[2] + F0[1]) / 2 + (F0[2] - F0[1]) / 2 * math.cos((b[3] * fs - i) / ((b[3] - b[1]) * fs) * math.pi)
        else:
            f0 = (F0[3] + F0[2]) / 2 + (F0[3] - F0[2]) / 2 * math.cos((b[6] * fs - i) / ((b[6] - b[3]) * fs) * math.pi)
        s = shapes4
        if i <= b[0] * fs:
            cur = np.array(s[0])
        elif i <= b[1] * fs:
            cur = interp(s[0], s[1], b[0] * fs, b[1] * fs, i)
        elif i <= b[2] * fs:
            cur = np.array(s[1])
        elif i <= b[3] * fs:
            cur = interp(s[1], s[2], b[2] * fs, b[3] * fs, i)
        elif i <= b[4] * fs:
            cur = np.array(s[2])
        elif i <= b[5] * fs:
            cur = interp(s[2], s[3], b[4] * fs, b[5] * fs, i)
        elif i <= b[6] * fs:
            cur = np.array(s[3])
        if i > (total - 0.1) * fs:
            pressure = -P / 2 * math.cos((total * fs - i) / (total - 0.1 * fs) * math.pi) + P / 2
        f0s.append(f0)
        prs.append(pressure)
        params.append(cur.copy())
    return np.array(f0s), np.array(prs), np.array(params)


def _vcv(v="a:", c="b"):
    sh = default_shapes()
    return np.stack([sh[v], sh[f"({v[0]}){c}({v[0]}):"], sh[v], sh[v]])


@pytest.mark.parametrize("fs,timing", [(44100.0, None), (22050.0, None), (44100.0, SHORT),
                                       (22050.0, {"stationary_s": [0.03, 0.0, 0.1, 0.07],
                                                  "transition_s": [0.02, 0.04, 0.0]})])
def test_trajectory_restatement_vs_python_statements(oracle, fs, timing):
    s4 = _vcv("i:", "g")
    cfg = oracle.target_cfg(timing)
    st, tr = list(cfg.stationary_s), list(cfg.transition_s)
    f0, pr, par = _python_trajectory(s4, fs, st, tr)
    fr = oracle.target_frames(s4, fs, timing)
    assert fr.size == f0.size + 1 == oracle.target_num_samples(fs, timing) + 1
    assert np.array_equal(fr["glottis"][1:, 0], f0)
    assert np.array_equal(fr["glottis"][1:, 1], pr)
    assert np.all(fr["glottis"][1:, 2:] == np.array([0.01, 0.01, 0.0, -40.0]))
    # the tube of sample i is the area function of its parameters (spot checks + every boundary)
    idx = sorted(set(range(0, f0.size, 97)) | {f0.size - 1} |
                 {int(x) for x in np.flatnonzero(np.any(np.diff(par, axis=0) != 0, axis=1))[:50]})
    for i in idx:
        want = oracle.af_to_frame(par[i])
        assert np.array_equal(fr[i + 1]["area_cm2"], want["area_cm2"]), i
        assert np.array_equal(fr[i + 1]["articulator"], want["articulator"]), i
        assert fr[i + 1]["teeth_position_cm"] == par[i][12]
    # frame 0: init()'s schwa latch with reset()'s glottis parameters
    schwa = [2.0, 1.0, 1.0, 3.02, 5.609, 1.0, 5.92, 2.879, 1.0, 8.48, 4.238, 1.0, 15.31, 0.701, 16.44, 1.65]
    assert np.array_equal(fr[0]["area_cm2"], oracle.af_to_frame(schwa)["area_cm2"])
    assert list(fr[0]["glottis"]) == [120.0, 10000.0, 0.01, 0.01, 0.0, -40.0]
    assert np.all(fr["velum_opening_cm2"] == 0.0)


def test_trajectory_shape_of_pressure_and_f0(oracle):
    fs = 44100.0
    fr = oracle.target_frames(_vcv(), fs)
    p = fr["glottis"][1:, 1]
    assert np.all(p[: int(0.05 * fs)] == 0.0)              # 50 ms silence
    assert p[int(0.1 * fs) + 10] == p[int(0.3 * fs)]         # held after the fade-in
    assert abs(p[int(0.3 * fs)] - 8000.0) < 0.01
    assert p[-1] < 1.0                                       # faded out at the end
    f = fr["glottis"][1:, 0]
    assert f[0] == 100.0 and abs(f[-1] - 80.0) < 1e-5


@pytest.mark.skipif(not os.path.exists("/root/reference/src/Backend"), reason="reference sources absent")
def test_target_sequence_synthesis_vs_reference(oracle):
    """Hop-1 synthesis of the trajectory (the reference's n = 1 calls) through the reference
    build equals the restatement bit for bit."""
    from oracle_lib import RefLib
    try:
        ref = RefLib()
    except FileNotFoundError:
        pytest.skip("reference build not available")
    for fs, (v, c), seed in ((44100.0, ("a:", "b"), 1), (22050.0, ("u:", "g"), 7)):
        fr = oracle.target_frames(_vcv(v, c), fs, SHORT)
        x = oracle.utterance(fr, 1, seed, fs)
        y = ref.utterance(fr, 1, seed, fs)
        assert np.array_equal(x, y)
        assert np.abs(x).max() > 1e-4


def test_golden_target_sequences(oracle, golden_dir):
    g = np.load(os.path.join(golden_dir, "target_seq.npz"), allow_pickle=False)
    timing = {"stationary_s": g["stationary_s"], "transition_s": g["transition_s"]}
    for k in range(g["targets"].shape[0]):
        s4 = g["shapes"][g["targets"][k]]
        y = oracle.target_sequence(s4, int(g["seeds"][k]), float(g["fs"]), timing)
        assert np.array_equal(y, g["out"][k]), k


# ---- GPU ----------------------------------------------------------------------------------

def _rms(a, b):
    return float(np.sqrt(np.mean((a - b) ** 2)))


@pytest.mark.gpu
def test_gpu_target_sequences_vs_golden(golden_dir):
    from areafunctionsynthesis_amd.synthesizer import Context
    g = np.load(os.path.join(golden_dir, "target_seq.npz"), allow_pickle=False)
    timing = {"stationary_s": g["stationary_s"], "transition_s": g["transition_s"]}
    ctx = Context(float(g["fs"]))
    # every golden row, plus repeats (the trajectory is built once per distinct sequence)
    targets = np.concatenate([g["targets"], g["targets"][:2]])
    seeds = np.concatenate([g["seeds"], g["seeds"][:2]]).astype(np.uint32)
    y, rep = ctx.play_target_sequences(g["shapes"], targets, timing, seeds=seeds, report=True)
    assert y.shape == (targets.shape[0], g["out"].shape[1])
    assert rep["nonfinite_utterances"] == 0
    for k in range(g["out"].shape[0]):
        assert np.abs(y[k, :2048] - g["out"][k, :2048]).max() <= 1e-9, k
        assert _rms(y[k], g["out"][k]) < 1e-4, k
    n = g["out"].shape[0]
    assert np.array_equal(y[n:], y[:2])


@pytest.mark.gpu
def test_gpu_target_sequence_default_timing_vs_oracle(oracle):
    """The reference's full playTargetSequence timing at 44.1 kHz (30870 samples), batched over
    the 15 VCV sequences with repeats; seeds per utterance."""
    from areafunctionsynthesis_amd.synthesizer import Context
    sh = default_shapes()
    names = sorted(sh)
    shapes = np.stack([sh[n] for n in names])
    pick = []
    for v in ("a:", "e:", "i:", "o:", "u:"):
        for c in ("b", "d", "g"):
            pick.append([names.index(v), names.index(f"({v[0]}){c}({v[0]}):"), names.index(v), names.index(v)])
    targets = np.array(pick * 3, dtype=np.int32)
    B = targets.shape[0]
    ctx = Context(44100.0)
    y = ctx.play_target_sequences(shapes, targets, seeds=np.arange(1, B + 1, dtype=np.uint32))
    assert y.shape == (B, ctx.target_sequence_samples())
    for u in (0, 7, 14, 15, 44):
        x = oracle.target_sequence(shapes[targets[u]], u + 1, 44100.0)
        assert np.abs(y[u, :2048] - x[:2048]).max() <= 1e-9, u
        assert _rms(y[u], x) < 1e-4, u
    assert not np.array_equal(y[0], y[15])  # same sequence, different seed


@pytest.mark.gpu
def test_gpu_target_sequence_equals_frames_path(oracle):
    """afs_play_target_sequences == afs_synthesize(oracle trajectory frames, hop 1): the GPU
    trajectory generator against the restatement through the same synthesis kernel."""
    from areafunctionsynthesis_amd.synthesizer import Context
    ctx = Context(22050.0)
    s4 = _vcv("o:", "d")
    y = ctx.play_target_sequences(s4, np.array([[0, 1, 2, 3]], dtype=np.int32), SHORT, seeds=np.array([5], np.uint32))
    fr = oracle.target_frames(s4, 22050.0, SHORT)
    z = ctx.synthesize(fr[None, :], 1, seeds=np.array([5], np.uint32))
    assert np.abs(y[0, :2048] - z[0, :2048]).max() <= 1e-9
    assert _rms(y[0], z[0]) < 1e-4


@pytest.mark.gpu
def test_gpu_target_sequence_errors():
    from areafunctionsynthesis_amd._native import AfsError
    from areafunctionsynthesis_amd.synthesizer import Context
    ctx = Context(22050.0)
    s4 = _vcv()
    with pytest.raises(AfsError):
        ctx.play_target_sequences(s4, np.array([[0, 1, 2, 4]], dtype=np.int32))
    with pytest.raises(ValueError):
        ctx.play_target_sequences(s4, np.array([0, 1, 2, 3], dtype=np.int32))
