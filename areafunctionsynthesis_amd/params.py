"""Area-function shape tables (the ``.params`` format) and the 16 model parameters.

``.params`` is the reference's shape-list format: two header lines, then one line per
shape, ``name`` followed by the 16 parameters separated by two spaces
(``src/Frontend/MainWindow.cpp:137-237``, read at ``:193-237``, written at
``:137-190``).  Parameter order is ``OneDimAreaFunction::ParamIndex``
(``src/Backend/OneDimAreaFunction.h:34-43``).
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass
from typing import Dict, Iterable, List

import numpy as np

PARAM_NAMES = (
    "Llar_cm", "Alar_cm2", "powLar", "xp_cm", "Ap_cm2", "powP", "xc_cm", "Ac_cm2",
    "powC", "xa_cm", "Aa_cm2", "powA", "xin_cm", "Ain_cm2", "Lvt_cm", "Alip_cm2",
)
NUM_AF_PARAMS = 16
(LLAR_CM, ALAR_CM2, POWLAR, XP_CM, AP_CM2, POWP, XC_CM, AC_CM2, POWC, XA_CM, AA_CM2,
 POWA, XIN_CM, AIN_CM2, LVT_CM, ALIP_CM2) = range(16)

_HEADER0 = "Parameters of one dimensional area functions for SecondVoicePc."
_HEADER1 = "Label " + "  ".join(PARAM_NAMES)

DATA_DIR = os.path.join(os.path.dirname(__file__), "data")


@dataclass
class Shape:
    name: str
    params: np.ndarray  # (16,) float64


def read_params(path: str) -> List[Shape]:
    """Parse a ``.params`` file (MainWindow::loadAfParamsList semantics)."""
    with open(path, "r", encoding="utf-8", errors="replace") as fh:
        lines = fh.read().splitlines()
    shapes = []
    for ln in lines[2:]:
        tok = ln.split()
        if not tok:
            continue
        vals = [float(t) for t in tok[1:1 + NUM_AF_PARAMS]]
        vals += [0.0] * (NUM_AF_PARAMS - len(vals))
        shapes.append(Shape(tok[0], np.asarray(vals, dtype=np.float64)))
    return shapes


def write_params(path: str, shapes: Iterable[Shape]) -> None:
    """Write shapes in the reference's format (``%f`` values, two-space separator)."""
    out = [_HEADER0, _HEADER1]
    for s in shapes:
        out.append(s.name + "  " + "  ".join("%f" % v for v in s.params))
    with open(path, "w", encoding="utf-8") as fh:
        fh.write("\n".join(out) + "\n")


def default_shapes() -> Dict[str, np.ndarray]:
    """The reference's default shape table (51 shapes), bundled as JSON."""
    with open(os.path.join(DATA_DIR, "shapes.json"), "r", encoding="utf-8") as fh:
        doc = json.load(fh)
    return {s["name"]: np.asarray(s["params"], dtype=np.float64) for s in doc["shapes"]}


# Vowel rows used by BASELINE config 2 (Default.params:3-31 long vowels and :35-42).
VOWELS = ("a:", "e:", "i:", "o:", "u:", "E:", "2:", "y:", "I", "E", "a", "O", "9", "Y", "U", "@")
FRICATIVES = ("s", "f", "z", "S", "Z", "x", "C", "R", "v")


def clamp_monotonic(p: np.ndarray) -> np.ndarray:
    """Monotonicity / non-negative-exponent clamps of
    OneDimAreaFunction::calculateParameter (OneDimAreaFunction.cpp:192-230)."""
    p = np.array(p, dtype=np.float64, copy=True)
    for a, b in ((XP_CM, LLAR_CM), (XC_CM, XP_CM), (XA_CM, XC_CM), (XIN_CM, XA_CM), (LVT_CM, XIN_CM)):
        p[..., a] = np.where(p[..., a] < p[..., b], p[..., b], p[..., a])
    for e in (POWLAR, POWP, POWC, POWA):
        p[..., e] = np.where(p[..., e] < 0, 0.0, p[..., e])
    return p
