"""The CPU emulator of the tree kernel and the oracle restatement under AddressSanitizer and
UndefinedBehaviorSanitizer (the tree kernel addresses its LDS block through u16
byte offsets in the section and step records, so a wrong offset would corrupt state silently;
the emulator runs the same phase code with the same records).  One executable
(tests/cpp/sanitize_main.cpp) per test module; each case must run clean (any report aborts it:
-fno-sanitize-recover) and the two outputs must agree as in test_tree_emu.py.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

from areafunctionsynthesis_amd.frames import DEFAULT_GLOTTIS, FRAME_DTYPE
from areafunctionsynthesis_amd.params import default_shapes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "areafunctionsynthesis_amd", "csrc")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]
TOL = 1e-9


@pytest.fixture(scope="module")
def sanitized(tmp_path_factory):
    if not shutil.which("g++") or not shutil.which("gcc"):
        pytest.skip("no host compiler")
    d = tmp_path_factory.mktemp("san")
    oracle_o = str(d / "afs_oracle.o")
    subprocess.check_call(["gcc", "-std=c11", "-O1", "-g", "-c", *SAN, "-I", os.path.join(ROOT, "oracle"),
                           os.path.join(ROOT, "oracle", "afs_oracle.c"), "-o", oracle_o])
    exe = str(d / "sanitize_main")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", *SAN, "-ffp-contract=off", "-fno-strict-aliasing",
                           "-Wno-unknown-pragmas", "-I", CSRC, "-I", os.path.join(ROOT, "oracle"),
                           os.path.join(ROOT, "tests", "cpp", "sanitize_main.cpp"),
                           os.path.join(ROOT, "tests", "emu", "tree_emu.cpp"), os.path.join(CSRC, "afs_tables.cpp"),
                           oracle_o, "-o", exe])
    return exe


def _run(exe, tmp_path, frames, hop, seed, fs, opt):
    from oracle_lib import OPTION_DEFAULTS
    o = dict(OPTION_DEFAULTS, **opt)
    iopt = np.array([o[k] for k in ("turbulence_losses", "soft_walls", "generate_noise_sources", "radiation_from_skin",
                                    "piriform_fossa", "inner_length_corrections", "transvelar_coupling",
                                    "glottis_loss", "glottis_model")], np.int32)
    src, dst = tmp_path / "in.bin", tmp_path / "out.bin"
    with open(src, "wb") as fh:
        fh.write(np.array([len(frames), hop], np.int32).tobytes())
        fh.write(np.array([seed], np.uint32).tobytes())
        fh.write(np.array([fs], np.float64).tobytes())
        fh.write(iopt.tobytes())
        fh.write(np.array([o["flow_separation_area_ratio"]], np.float64).tobytes())
        fh.write(np.ascontiguousarray(frames, FRAME_DTYPE).tobytes())
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, str(src), str(dst)], capture_output=True, text=True, env=env)
    assert r.returncode == 0 and "runtime error" not in r.stderr, r.stderr[-3000:]
    T = (len(frames) - 1) * hop
    both = np.fromfile(dst, np.float64)
    return both[:T], both[T:]


CASES = {
    "vowels": ([("a:", 0.0), ("i:", 0.0), ("u:", 0.0)], {}),
    "fricatives+velum": ([("s", 1.0), ("S", 1.0), ("f", 0.5), ("x", 1.0)], {}),
    "vcv-closure": ([("a:", 0.0), ("(a)b(a):", 0.0), ("(a)g(a):", 0.3), ("a:", 0.0)], {}),
    "options": ([("z", 0.5), ("a:", 0.5)], {"transvelar_coupling": 1, "glottis_loss": 2, "piriform_fossa": 1}),
    "two-mass": ([("i:", 0.2), ("C", 0.2)], {"glottis_model": 1}),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_emulator_and_oracle_clean_under_asan_ubsan(sanitized, oracle, tmp_path, case):
    seq, opt = CASES[case]
    sh = default_shapes()
    frames = np.stack([oracle.af_to_frame(sh[n]) for n, _ in seq])
    frames["velum_opening_cm2"] = [v for _, v in seq]
    frames["glottis"] = DEFAULT_GLOTTIS
    if opt.get("glottis_model"):  # control 5 is the two-mass model's damping factor
        frames["glottis"][:, 5] = 1.2
    frames["laterality"][:, 28:33] = 0.15
    x, y = _run(sanitized, tmp_path, frames, 331, 7, 44100.0, opt)
    assert np.abs(x - y).max() <= TOL
