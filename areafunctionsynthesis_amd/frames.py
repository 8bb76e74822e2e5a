"""Frame records: the per-call inputs of ``Synthesizer::synthesizeSignalTds``.

One frame is the dynamic part of a ``Tube`` (the 40 pharynx/mouth sections, the
incisor position and the velum opening; ``src/Backend/Tube.h:33-108``) plus the six
``TriangularGlottis`` control parameters (``src/Backend/TriangularGlottis.h:26-35``).
The byte layout is ``afs_frame`` of ``include/afs.h`` (1072 bytes).

A batch is ``frames[B, F]``: utterance ``u`` is synthesised as the reference would
with one latch call on ``frames[u, 0]`` followed by ``F-1`` calls of ``hop`` samples
(``src/Backend/Synthesizer.cpp:522-532`` and ``:557-629``).
"""
from __future__ import annotations

import enum

import numpy as np

NUM_PM_SECTIONS = 40          # Tube::NUM_PHARYNX_MOUTH_SECTIONS (Tube.h:56-58)
NUM_GLOTTIS_PARAMS = 6        # TriangularGlottis::NUM_CONTROL_PARAMS
MIN_AREA_CM2 = 0.1e-2         # Tube::MIN_AREA_CM2 (Tube.cpp:12)

FRAME_DTYPE = np.dtype(
    [
        ("area_cm2", "<f8", (NUM_PM_SECTIONS,)),
        ("length_cm", "<f8", (NUM_PM_SECTIONS,)),
        ("laterality", "<f8", (NUM_PM_SECTIONS,)),
        ("teeth_position_cm", "<f8"),
        ("velum_opening_cm2", "<f8"),
        ("glottis", "<f8", (NUM_GLOTTIS_PARAMS,)),
        ("articulator", "u1", (NUM_PM_SECTIONS,)),
        ("pad", "u1", (8,)),
    ],
    align=False,
)
assert FRAME_DTYPE.itemsize == 1072


class Articulator(enum.IntEnum):
    """Tube::Articulator (Tube.h:24-32)."""

    VOCAL_FOLDS = 0
    TONGUE = 1
    LOWER_INCISORS = 2
    LOWER_LIP = 3
    OTHER_ARTICULATOR = 4


class GlottisParam(enum.IntEnum):
    """TriangularGlottis::ControlParamIndex (TriangularGlottis.h:26-35)."""

    FREQUENCY = 0
    PRESSURE = 1
    REST_DISP_1 = 2
    REST_DISP_2 = 3
    ARY_AREA = 4
    ASPIRATION_STRENGTH = 5


# Neutral control values (TriangularGlottis.cpp:17-25) with the lung pressure the
# real-time caller uses (Synthesizer.cpp:905).
DEFAULT_GLOTTIS = (120.0, 8000.0, 0.01, 0.01, 0.0, -40.0)


def empty_frames(*shape: int) -> np.ndarray:
    """Zeroed frame array of the given shape."""
    return np.zeros(shape, dtype=FRAME_DTYPE)


def set_glottis(frames: np.ndarray, f0=None, pressure=None, rest1=None, rest2=None,
                ary=None, aspiration_db=None) -> None:
    """Write glottis control values (broadcasting) into ``frames``."""
    g = frames["glottis"]
    for idx, val in enumerate((f0, pressure, rest1, rest2, ary, aspiration_db)):
        if val is not None:
            g[..., idx] = val
