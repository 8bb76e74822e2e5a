"""The wave-pair kernels (tree_kernel.h tree_pair_body / tree_pair64_body): the phases of each group of
utterances split between a DYN and a STAT wave that meet at workgroup barriers.  The 64-lane pairs
(`tree_pair64_kernel`, batches up to the SIMD count) and the 64-lane one-wave kernel
(`tree_synth_kernel<.., 64>`, larger batches forced to 64 lanes) are both in the default build, so
the pairs are checked against the one-wave form bit for bit here; the 16-lane pairs' one-wave form is
an A/B build (AFS_PAIR=0; tools/lib_equal.py, profiles/r06_pair_ab.txt r06m)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_kernel_names():
    from areafunctionsynthesis_amd.synthesizer import Context
    auto = Context(44100.0, solver="tree")
    forced = Context(44100.0, solver="tree", lanes=64)
    try:
        assert auto.synthesis_kernel(1) == "tree_pair64_kernel"
        assert auto.synthesis_kernel(1024) == "tree_pair64_kernel"
        assert auto.synthesis_kernel(1025) == "tree_pair_kernel"
        assert auto.synthesis_kernel(65536) == "tree_pair_kernel"
        assert forced.synthesis_kernel(1024) == "tree_pair64_kernel"
        assert forced.synthesis_kernel(2048) == "tree_synth_kernel"
    finally:
        auto.close()
        forced.close()


@pytest.mark.parametrize("workload", ["static_vowels", "fricatives"])
def test_voice_pairs_equal_one_wave_bitwise(workload, parity_report):
    """2048 utterances forced to 64 lanes run one wave per utterance; the first 256 alone run as wave
    pairs: the same audio bit for bit, and the same rand() counts."""
    from areafunctionsynthesis_amd import workloads
    from areafunctionsynthesis_amd.synthesizer import Context
    ctx = Context(44100.0, solver="tree", lanes=64)
    try:
        w = getattr(workloads, workload)(2048, seconds=0.05, fs=44100.0)
        frames = workloads.build_frames(w, ctx.af_to_frames)
        assert ctx.synthesis_kernel(2048) == "tree_synth_kernel"
        one = ctx.synthesize(frames, w.hop, seeds=w.seeds)
        d_one = ctx.rng_draws(2048)[:256]
        assert ctx.synthesis_kernel(256) == "tree_pair64_kernel"
        pair = ctx.synthesize(frames[:256], w.hop, seeds=w.seeds[:256])
        d_pair = ctx.rng_draws(256)
    finally:
        ctx.close()
    same = bool(np.array_equal(one[:256], pair))
    parity_report.append(
        f"voice pairs vs one wave per utterance (64 lanes, {workload}, 256 utterances x {w.samples_per_utterance} "
        f"samples): bitwise {same}, max |diff| {np.abs(one[:256] - pair).max():.3e}; rand() counts equal: "
        f"{bool(np.array_equal(d_one, d_pair))}")
    assert np.isfinite(pair).all()
    assert same
    assert np.array_equal(d_one, d_pair)
