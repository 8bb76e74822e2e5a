"""Synthetic utterance batches for the BASELINE.json configurations.

Each generator returns area-function parameters and glottis/velum controls per frame;
:func:`build_frames` turns them into ``afs_frame`` records with the GPU area-function
kernel (``Context.af_to_frames``) or any other ``params -> frames`` function.

* ``static_vowels``  config 2 / 4: shapes drawn from the 16 vowel rows of the default
  shape table, every parameter jittered by N(0, 2 %), monotonicity-clamped
  (OneDimAreaFunction.cpp:192-230), f0 ~ U[90, 180] Hz, lung pressure ~ U[6000, 10000]
  dPa, rest displacement 0.01 cm, aspiration -40 dB, velum closed.
* ``vcv``            config 3: V-C-V target sequences timed like
  Synthesizer::playTargetSequence (Synthesizer.cpp:1299-1422) and sampled at 100 Hz
  frames (Synthesizer::FRAME_RATE_HZ, Synthesizer.h:58).
* ``vcv_targets``    config 3 as the reference actually plays it: four target shapes per
  utterance for ``Context.play_target_sequences`` (per-sample tubes, hop 1).
* ``fricatives``     config 5: fricative shapes with the velum open 1.0 cm^2
  (the GUI's default port area, MainPage.cpp:127-131), so the noise sources and the
  nasal side branch are active.
Utterance ``u`` is seeded ``u + 1`` (srand per utterance) and draws its shape and
glottis settings from its own generator (SeedSequence [build seed, u]), so a shard built
with ``first_utterance`` holds exactly the rows of the full batch and the audio does not
depend on the GPU count.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from .frames import FRAME_DTYPE
from .params import FRICATIVES, VOWELS, clamp_monotonic, default_shapes

BUILD_SEED = 0xAF5


@dataclass
class Workload:
    name: str
    params: np.ndarray    # [B, F, 16]
    glottis: np.ndarray   # [B, F, 6]
    velum: np.ndarray     # [B, F]
    hop: int
    fs: float
    seeds: np.ndarray     # [B] uint32

    @property
    def batch(self) -> int:
        return self.params.shape[0]

    @property
    def num_frames(self) -> int:
        return self.params.shape[1]

    @property
    def samples_per_utterance(self) -> int:
        return (self.num_frames - 1) * self.hop


def _seeds(B: int, first: int) -> np.ndarray:
    return (np.arange(B, dtype=np.uint64) + 1 + first).astype(np.uint32)


def _rows(seed: int, first: int, B: int, n_choices: int):
    """Per-utterance draws: shape index, 16 N(0,1) jitters, U[0,1) x 2 (global index u)."""
    pick = np.empty(B, np.int64)
    jit = np.empty((B, 16))
    uni = np.empty((B, 2))
    for k in range(B):
        g = np.random.default_rng([seed, first + k])
        pick[k] = g.integers(0, n_choices)
        jit[k] = g.standard_normal(16)
        uni[k] = g.random(2)
    return pick, jit, uni


def static_vowels(B: int, seconds: float = 1.0, fs: float = 44100.0, frame_rate: float = 100.0,
                  first_utterance: int = 0, seed: int = BUILD_SEED) -> Workload:
    """Config 2/4 generator.  ``first_utterance`` offsets the per-utterance draws so a
    shard of a larger batch gets exactly the rows the full batch would give it."""
    shapes = default_shapes()
    base = np.stack([shapes[v] for v in VOWELS])
    hop = int(round(fs / frame_rate))
    F = int(round(seconds * fs / hop)) + 1
    pick, jit, uni = _rows(seed, first_utterance, B, len(VOWELS))
    f0 = 90.0 + 90.0 * uni[:, 0]
    pl = 6000.0 + 4000.0 * uni[:, 1]
    p = clamp_monotonic(base[pick] * (1.0 + 0.02 * jit))
    params = np.repeat(p[:, None, :], F, axis=1)
    glottis = np.zeros((B, F, 6))
    glottis[..., 0] = f0[:, None]
    glottis[..., 1] = pl[:, None]
    glottis[..., 2] = 0.01
    glottis[..., 3] = 0.01
    glottis[..., 4] = 0.0
    glottis[..., 5] = -40.0
    return Workload("static_vowels", params, glottis, np.zeros((B, F)), hop, fs, _seeds(B, first_utterance))


def fricatives(B: int, seconds: float = 1.0, fs: float = 44100.0, frame_rate: float = 100.0,
               velum_cm2: float = 1.0, first_utterance: int = 0, seed: int = BUILD_SEED + 5) -> Workload:
    shapes = default_shapes()
    base = np.stack([shapes[v] for v in FRICATIVES])
    hop = int(round(fs / frame_rate))
    F = int(round(seconds * fs / hop)) + 1
    pick, jit, uni = _rows(seed, first_utterance, B, len(FRICATIVES))
    f0 = 90.0 + 90.0 * uni[:, 0]
    p = clamp_monotonic(base[pick] * (1.0 + 0.02 * jit))
    params = np.repeat(p[:, None, :], F, axis=1)
    glottis = np.zeros((B, F, 6))
    glottis[..., 0] = f0[:, None]
    glottis[..., 1] = 8000.0
    glottis[..., 2] = 0.01
    glottis[..., 3] = 0.01
    glottis[..., 5] = -40.0
    return Workload("fricatives", params, glottis, np.full((B, F), velum_cm2), hop, fs, _seeds(B, first_utterance))


def _cos_interp(p0, p1, t0, t1, tx):
    # Synthesizer::interpolateParameters, Synthesizer.cpp:1286-1294
    return (p1 - p0) / 2 * math.cos((t1 - tx) / (t1 - t0) * math.pi) + (p1 + p0) / 2


def vcv(B: int, fs: float = 44100.0, frame_rate: float = 100.0, first_utterance: int = 0,
        seed: int = BUILD_SEED + 3, stationary=(0.2, 0.05, 0.2, 0.1), transition=(0.05, 0.05, 0.05)) -> Workload:
    """V-(V)C(V)-V-V target sequences with playTargetSequence's timing, F0 contour and
    lung-pressure fades, evaluated at the frame instants."""
    shapes = default_shapes()
    vowels = ("a:", "e:", "i:", "o:", "u:")
    cons = ("b", "d", "g")
    hop = int(round(fs / frame_rate))
    bnd = np.cumsum([stationary[0], transition[0], stationary[1], transition[1], stationary[2],
                     transition[2], stationary[3]])
    total_s = float(bnd[-1])
    F = int(math.floor(total_s * fs / hop)) + 1
    pick, _, _ = _rows(seed, first_utterance, B, len(vowels) * len(cons))
    vi, ci = pick // len(cons), pick % len(cons)
    f0s = (100.0, 115.0, 105.0, 80.0)  # Synthesizer.cpp:1311
    P = 8000.0
    params = np.zeros((B, F, 16))
    glottis = np.zeros((B, F, 6))
    glottis[..., 2] = 0.01
    glottis[..., 3] = 0.01
    glottis[..., 5] = -40.0
    for u in range(B):
        v = vowels[vi[u]]
        c = cons[ci[u]]
        seq = [shapes[v], shapes[f"({v[0]}){c}({v[0]}):"], shapes[v], shapes[v]]
        for k in range(F):
            i = k * hop
            t = [b * fs for b in bnd]
            if i <= t[0]:
                p = seq[0]
            elif i <= t[1]:
                p = _cos_interp(seq[0], seq[1], t[0], t[1], i)
            elif i <= t[2]:
                p = seq[1]
            elif i <= t[3]:
                p = _cos_interp(seq[1], seq[2], t[2], t[3], i)
            elif i <= t[4]:
                p = seq[2]
            elif i <= t[5]:
                p = _cos_interp(seq[2], seq[3], t[4], t[5], i)
            else:
                p = seq[3]
            params[u, k] = p
            if i < t[1]:
                f0 = (f0s[0] + f0s[1]) / 2 + (f0s[1] - f0s[0]) / 2 * math.cos((t[1] - i) / t[1] * math.pi)
            elif i < t[3]:
                f0 = (f0s[2] + f0s[1]) / 2 + (f0s[2] - f0s[1]) / 2 * math.cos((t[3] - i) / (t[3] - t[1]) * math.pi)
            else:
                f0 = (f0s[3] + f0s[2]) / 2 + (f0s[3] - f0s[2]) / 2 * math.cos((t[6] - i) / (t[6] - t[3]) * math.pi)
            if i < 0.05 * fs:
                pr = 0.0
            elif i < 0.1 * fs:
                pr = P / 2 * math.cos((0.1 * fs - i) / (0.05 * fs) * math.pi) + P / 2
            elif i > (total_s - 0.1) * fs:
                pr = -P / 2 * math.cos((total_s * fs - i) / (0.1 * fs) * math.pi) + P / 2
            else:
                pr = P
            glottis[u, k, 0] = f0
            glottis[u, k, 1] = pr
    return Workload("vcv", params, glottis, np.zeros((B, F)), hop, fs, _seeds(B, first_utterance))


VCV_VOWELS = ("a:", "e:", "i:", "o:", "u:")
VCV_CONSONANTS = ("b", "d", "g")


def vcv_targets(B: int, first_utterance: int = 0, seed: int = BUILD_SEED + 3):
    """Config 3 for Context.play_target_sequences: utterance u plays the targets
    V, (V)C(V):, V, V (the reference's four-shape playTargetSequence) for V, C drawn per
    utterance.  Returns (shapes[S, 16], targets[B, 4] int32, seeds[B] uint32)."""
    sh = default_shapes()
    names = list(VCV_VOWELS) + [f"({v[0]}){c}({v[0]}):" for v in VCV_VOWELS for c in VCV_CONSONANTS]
    shapes = np.stack([sh[n] for n in names])
    pick, _, _ = _rows(seed, first_utterance, B, len(VCV_VOWELS) * len(VCV_CONSONANTS))
    vi, ci = pick // len(VCV_CONSONANTS), pick % len(VCV_CONSONANTS)
    cons_row = len(VCV_VOWELS) + vi * len(VCV_CONSONANTS) + ci
    targets = np.stack([vi, cons_row, vi, vi], axis=1).astype(np.int32)
    return shapes, targets, _seeds(B, first_utterance)


def build_frames(w: Workload, af_to_frames) -> np.ndarray:
    """Frames[B, F] from a workload; ``af_to_frames(params[N,16]) -> frames[N]``."""
    B, F = w.batch, w.num_frames
    if (w.params == w.params[:, :1, :]).all():
        # static utterances: one parameter row each (the 64k batch: 65536 rows to sort, not 6.6 M)
        uniq, inv = np.unique(w.params[:, 0, :], axis=0, return_inverse=True)
        fu = af_to_frames(uniq)
        frames = np.repeat(fu[inv.reshape(-1)][:, None], F, axis=1)
    else:
        # convert unique rows only
        uniq, inv = np.unique(w.params.reshape(B * F, 16), axis=0, return_inverse=True)
        fu = af_to_frames(uniq)
        frames = fu[inv.reshape(-1)].reshape(B, F).copy()
    frames["velum_opening_cm2"] = w.velum
    frames["glottis"] = w.glottis
    return frames
