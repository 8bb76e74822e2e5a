"""include/afs_synthesizer.hpp: the C++ adapter a reference-side caller uses.

CPU: the Tube -> afs_frame conversion round-trips bit for bit and errors surface as
afs::Error.  GPU: the adapter, driven like Synthesizer::synthesizeSignalTds (latch, then one
call per frame), matches the oracle.
"""
import os
import subprocess

import numpy as np
import pytest

from areafunctionsynthesis_amd.frames import DEFAULT_GLOTTIS, FRAME_DTYPE
from areafunctionsynthesis_amd.params import default_shapes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "areafunctionsynthesis_amd")


@pytest.fixture(scope="module")
def adapter_bin(tmp_path_factory):
    from areafunctionsynthesis_amd import _native
    _native.load()  # builds libafs.so if needed
    exe = str(tmp_path_factory.mktemp("adapter") / "adapter_main")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "adapter_main.cpp"), "-L", PKG, "-lafs",
                           f"-Wl,-rpath,{PKG}", "-o", exe])
    return exe


def test_frame_from_tube_roundtrip(adapter_bin):
    out = subprocess.run([adapter_bin, "frames"], capture_output=True, text=True, check=True).stdout
    assert out.strip() == "frames-equal"


def test_missing_device_raises(adapter_bin):
    out = subprocess.run([adapter_bin, "nodevice"], capture_output=True, text=True, check=True).stdout
    assert out.strip() == "error 2"  # AFS_ERR_NO_DEVICE


@pytest.mark.gpu
def test_adapter_single_voice_vs_oracle(adapter_bin, oracle, tmp_path):
    f = oracle.af_to_frame(default_shapes()["s"])
    f["velum_opening_cm2"] = 0.5
    f["glottis"] = DEFAULT_GLOTTIS
    frames = np.repeat(f[None], 6)
    frames["glottis"][:, 0] = np.linspace(110, 130, 6)
    hop, fs, seed = 97, 22050.0, 4
    src = tmp_path / "in.bin"
    with open(src, "wb") as fh:
        fh.write(np.array([len(frames), hop], np.int32).tobytes())
        fh.write(np.array([fs], np.float64).tobytes())
        fh.write(np.array([seed], np.uint32).tobytes())
        fh.write(np.ascontiguousarray(frames, FRAME_DTYPE).tobytes())
    dst = tmp_path / "out.bin"
    subprocess.run([adapter_bin, "synth", str(src), str(dst), "x"], check=True, capture_output=True)
    y = np.fromfile(dst, np.float64)
    x = oracle.utterance(frames, hop, seed, fs)
    assert y.shape == x.shape == ((len(frames) - 1) * hop,)
    assert np.abs(y - x).max() <= 1e-9


@pytest.mark.gpu
def test_adapter_realtime_latency(adapter_bin, oracle, tmp_path, parity_report):
    """The real-time drop-in: one voice (TdsVoices<Tube>, batch 1) called like
    SynthesisThread (SynthesisThread.cpp:18-35) with 1102-sample chunks -- 50 ms of audio at
    22.05 kHz, the reference's buffer (Synthesizer.cpp:953, Synthesizer.h:63) -- for 100 calls
    (5.5 s of a gliding fricative).  Per call: the wall time, and in it the tube conversion and
    the K5 / K1 / K6 device times (HIP events); the rest is the host's copies, launches and waits.
    Bounds: the hard real-time one -- no call's wall time above the 50 ms of audio it makes (the first
    synthesis call included: afs_create loads the kernels' code objects, which HIP otherwise loads at
    their first launch) -- and, on the device time of a call (K5 + K1 + K6, HIP events: free of the
    host's scheduling jitter on a shared box), p99 below 6.0 ms -- 20 % under the reference core's
    time for the same 1102 samples (7.5 ms: 147 k samples/s per core, bench.py cpu_baseline); the voice
    kernel's wave pairs measured 5.2 ms.  The wall-time p99 is reported, not asserted."""
    f = oracle.af_to_frame(default_shapes()["s"])
    f["velum_opening_cm2"] = 0.2
    f["glottis"] = DEFAULT_GLOTTIS
    F = 101
    frames = np.repeat(f[None], F)
    frames["glottis"][:, 0] = 110 + 20 * np.sin(np.linspace(0, 6, F))
    hop, fs, seed = 1102, 22050.0, 9
    src = tmp_path / "in.bin"
    with open(src, "wb") as fh:
        fh.write(np.array([F, hop], np.int32).tobytes())
        fh.write(np.array([fs], np.float64).tobytes())
        fh.write(np.array([seed], np.uint32).tobytes())
        fh.write(np.ascontiguousarray(frames, FRAME_DTYPE).tobytes())
    dst = tmp_path / "ms.bin"
    subprocess.run([adapter_bin, "latency", str(src), str(dst), "x"], check=True, capture_output=True)
    t = np.fromfile(dst, np.float64).reshape(F, 5)[1:]  # (the first call latches the tube and makes no samples)
    ms, conv, k5, k1, k6 = t.T
    rest = ms - k5 - k1 - k6
    assert ms.shape == (F - 1,)
    p50, p99 = np.percentile(ms, 50), np.percentile(ms, 99)
    dev = k5 + k1 + k6
    d99 = np.percentile(dev, 99)
    w = int(np.argmax(ms))
    parity_report.append(
        f"real-time drop-in (TdsVoices<Tube>, batch 1, {hop}-sample calls @ {fs:g} Hz = {hop / fs * 1e3:.0f} ms of "
        f"audio per call, {F - 1} calls): wall time per call p50 {p50:.2f} ms p99 {p99:.2f} ms max {ms.max():.2f} ms "
        f"(reference core: 7.5 ms); device time (K5 + K1 + K6) p50 {np.median(dev):.2f} ms p99 {d99:.2f} ms; "
        f"per call (median) tube conversion {np.median(conv) * 1e3:.1f} us, K5 {np.median(k5):.3f} ms, K1 "
        f"{np.median(k1):.3f} ms, K6 {np.median(k6):.3f} ms, host copies / launches / waits {np.median(rest):.3f} ms; "
        f"slowest call (#{w + 1}): conversion {conv[w] * 1e3:.1f} us, K5 {k5[w]:.3f}, K1 {k1[w]:.3f}, K6 {k6[w]:.3f}, "
        f"host {rest[w]:.3f} ms")
    assert ms.max() < hop / fs * 1e3, (p50, p99, ms.max(), w, t[w])
    assert d99 < 6.0, (np.median(dev), d99)


REF_BACKEND = "/root/reference/src/Backend"
REF_TUBE_O = os.path.join(ROOT, "oracle", "_ref", "obj", "Tube.o")


@pytest.fixture(scope="module")
def tube_bin(tmp_path_factory):
    if not (os.path.isdir(REF_BACKEND) and os.path.exists(REF_TUBE_O)):
        pytest.skip("the reference's Tube (/root/reference + oracle/_ref) is not available here")
    exe = str(tmp_path_factory.mktemp("tube") / "tube_main")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-w", "-I", REF_BACKEND, "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "tube_main.cpp"), REF_TUBE_O, "-o", exe])
    return exe


def test_frame_from_reference_tube(tube_bin, oracle, tmp_path):
    """afs::frame_from_tube<Tube> on the reference's own Tube class, filled through
    Tube::setPharynxMouthGeometry / setVelumOpening (Tube.cpp:323-349, 402-416): the frame holds
    exactly what those setters store (areas and velum clamped at MIN_AREA_CM2 = 0.001, Tube.cpp:337,
    413), and that frame synthesizes bit for bit like the caller's original input."""
    sh = default_shapes()
    rng = np.random.default_rng(5)
    names = ["a:", "s", "i:", "(a)b(a):", "S", "u:", "f", "x"]
    frames = np.stack([oracle.af_to_frame(sh[n]) for n in names])
    frames["glottis"] = DEFAULT_GLOTTIS
    frames["velum_opening_cm2"] = [0.0, 1.0, 0.5, 1e-5, 0.25, 0.0, 2.0, 0.0005]
    frames["laterality"][:, 20:30] = rng.random((len(names), 10)) * 0.3
    frames["area_cm2"][2, 5] = 1e-6          # below MIN_AREA: the setter clamps
    frames["area_cm2"][4, 39] = 0.0
    src, dst = tmp_path / "in.bin", tmp_path / "out.bin"
    with open(src, "wb") as fh:
        fh.write(np.array([len(frames)], np.int32).tobytes())
        fh.write(np.ascontiguousarray(frames, FRAME_DTYPE).tobytes())
    out = subprocess.run([tube_bin, str(src), str(dst)], capture_output=True, text=True, check=True).stdout
    assert out.strip() == f"ok {len(frames)}"
    got = np.fromfile(dst, FRAME_DTYPE)
    want = frames.copy()
    want["area_cm2"] = np.maximum(want["area_cm2"], 0.001)
    want["velum_opening_cm2"] = np.maximum(want["velum_opening_cm2"], 0.001)
    assert got.tobytes() == np.ascontiguousarray(want, FRAME_DTYPE).tobytes()
    # the synthesis clamps exactly as the Tube does, so the caller's frame and the Tube's agree
    seq = np.stack([got[[0, 1, 3, 1]], frames[[0, 1, 3, 1]]])
    x = oracle.utterance(seq[0], 97, 3, 44100.0)
    y = oracle.utterance(seq[1], 97, 3, 44100.0)
    assert np.array_equal(x, y)
