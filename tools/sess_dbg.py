import os, sys, numpy as np
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), 'tests'))
import torch; torch.cuda.init()
from oracle_lib import Oracle
from areafunctionsynthesis_amd.frames import FRAME_DTYPE
from areafunctionsynthesis_amd.params import default_shapes
from areafunctionsynthesis_amd.synthesizer import Context, Synthesizer
oracle = Oracle(); sh = default_shapes()
B, F, hop = 3, 6, 150
frames = np.zeros((B, F), FRAME_DTYPE)
for u in range(B):
    for k in range(F):
        f = oracle.af_to_frame(sh[["a:", "(a)d(a):", "i:", "s"][(u + k) % 4]])
        f["glottis"] = [100 + 10 * k, 8000, 0.01, 0.01, 0, -40]
        frames[u, k] = f
seeds = np.array([3, 4, 5], np.uint32)
for dense in ("0", "1"):
    os.environ["AFS_PLAN_DENSE"] = dense
    ctx = Context(22050.0, solver="tree")
    y = ctx.synthesize(frames, hop, seeds=seeds)
    syn = Synthesizer(ctx, B, seeds)
    syn.synthesize_signal_tds(frames[:, 0], hop)
    parts = np.concatenate([syn.synthesize_signal_tds(frames[:, k], hop) for k in range(1, F)], axis=1)
    d = np.abs(parts - y)
    bad = np.argwhere(d > 0)
    print("dense", dense, "equal", np.array_equal(parts, y), "max", d.max(), "first diff", bad[:3].tolist() if len(bad) else None,
          "oracle maxdiff", max(np.abs(y[u] - oracle.utterance(frames[u], hop, int(seeds[u]), 22050.0)).max() for u in range(B)))
    syn.close(); ctx.close()
