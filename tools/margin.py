"""Parity margin of the tree kernel on the mixed 70-utterance batch of test_gpu_parity
(development tool): per-utterance max |gpu - oracle| over the first 2048 samples."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle_lib import Oracle  # noqa: E402

from areafunctionsynthesis_amd.frames import FRAME_DTYPE  # noqa: E402
from areafunctionsynthesis_amd.params import default_shapes  # noqa: E402
from areafunctionsynthesis_amd.synthesizer import Context  # noqa: E402


def main():
    oracle = Oracle()
    sh = default_shapes()
    names = ["a:", "i:", "u:", "e:", "o:", "s", "f", "x", "S", "(a)b(a):", "l", "C"]
    rng = np.random.default_rng(7)
    B, F, hop, fs = 70, 9, 256, 22050.0
    frames = np.zeros((B, F), FRAME_DTYPE)
    for u in range(B):
        for k in range(F):
            f = oracle.af_to_frame(sh[names[(u + k // 4) % len(names)]] * (1 + 0.01 * rng.standard_normal(16)))
            f["velum_opening_cm2"] = (0.0, 1.0)[u % 2]
            f["laterality"] = np.clip(rng.uniform(-0.5, 0.3, 40), 0, 1) if u % 5 == 0 else 0.0
            f["glottis"] = [rng.uniform(90, 180), rng.uniform(6000, 10000), 0.01, 0.01, 0.0, -40.0 + 20 * (u % 3)]
            frames[u, k] = f
    seeds = np.arange(1, B + 1, dtype=np.uint32)
    for solver in ("tree",):
        y = Context(fs, solver=solver).synthesize(frames, hop, seeds=seeds)
        errs = np.array([np.abs(y[u] - oracle.utterance(frames[u], hop, int(seeds[u]), fs)).max() for u in range(B)])
        q = np.quantile(errs, [0.5, 0.9, 1.0])
        print(f"{solver}: median {q[0]:.2e} p90 {q[1]:.2e} max {q[2]:.2e} (utterance {int(errs.argmax())})")


if __name__ == "__main__":
    main()
