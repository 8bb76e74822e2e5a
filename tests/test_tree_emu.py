"""CPU check of the cooperative tree kernel's decomposition (test-only host build of
csrc/tree_core.h, see tests/emu/tree_emu.cpp): lane ownership, LDS exchange and the
fill-free LDL^T schedule reproduce the oracle to rounding level, for any lane width."""
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
    run.lib = lib
    return run


def test_schedule_is_valid(emu):
    # build_tables verifies fill-freeness / round conflicts and reports -1 otherwise
    assert emu.lib.emu_tree_rounds(22050.0) == 16  # nested-dissection plan (afs_tables.cpp tree_schedule)


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
