"""16-bit PCM WAV files of synthesized utterances.

The reference's final audio format is the int16 ring ``Signal16`` filled by
``Synthesizer::synthesizeSegment`` (src/Backend/Synthesizer.cpp:955-973); the conversion
itself runs on the GPU (``Context.to_int16`` -> ``afs_to_int16``).  This module only frames
those int16 samples as canonical mono RIFF/WAVE files (44-byte header, little endian).
"""
from __future__ import annotations

import os
import struct
from typing import Sequence, Tuple

import numpy as np

HEADER_BYTES = 44


def wav_header(num_samples: int, sampling_rate_hz: int, channels: int = 1) -> bytes:
    """Canonical PCM header: RIFF size, fmt chunk (PCM, 16 bit), data chunk size."""
    if num_samples < 0 or sampling_rate_hz <= 0 or channels < 1:
        raise ValueError("bad WAV parameters")
    block = 2 * channels
    data = num_samples * block
    return (b"RIFF" + struct.pack("<I", 36 + data) + b"WAVE"
            + b"fmt " + struct.pack("<IHHIIHH", 16, 1, channels, sampling_rate_hz, sampling_rate_hz * block, block, 16)
            + b"data" + struct.pack("<I", data))


def _as_pcm(samples) -> np.ndarray:
    if hasattr(samples, "detach"):  # torch tensor (device or host)
        samples = samples.detach().cpu().numpy()
    x = np.asarray(samples)
    if x.dtype != np.int16:
        raise TypeError(f"WAV samples must be int16 (use Context.to_int16), got {x.dtype}")
    return np.ascontiguousarray(x.reshape(-1)).astype("<i2", copy=False)


def write_wav(path: str, samples, sampling_rate_hz: float) -> None:
    """Write one mono utterance of int16 samples."""
    pcm = _as_pcm(samples)
    with open(path, "wb") as f:
        f.write(wav_header(pcm.size, int(round(sampling_rate_hz))))
        f.write(pcm.tobytes())


def write_batch(directory: str, samples, sampling_rate_hz: float, names: Sequence[str] = None) -> list:
    """One file per row of an int16 [B, T] batch; returns the paths."""
    x = samples.detach().cpu().numpy() if hasattr(samples, "detach") else np.asarray(samples)
    if x.ndim != 2:
        raise ValueError("expected an int16 [B, T] batch")
    os.makedirs(directory, exist_ok=True)
    names = names if names is not None else [f"utt{b:06d}" for b in range(x.shape[0])]
    if len(names) != x.shape[0]:
        raise ValueError("one name per utterance")
    paths = []
    for b, name in enumerate(names):
        p = os.path.join(directory, f"{name}.wav")
        write_wav(p, x[b], sampling_rate_hz)
        paths.append(p)
    return paths


def read_wav(path: str) -> Tuple[np.ndarray, int]:
    """Read back a mono 16-bit PCM file written by :func:`write_wav` (int16 samples, rate)."""
    with open(path, "rb") as f:
        raw = f.read()
    if raw[:4] != b"RIFF" or raw[8:12] != b"WAVE":
        raise ValueError("not a RIFF/WAVE file")
    pos, fmt, data = 12, None, None
    while pos + 8 <= len(raw):
        cid, size = raw[pos:pos + 4], struct.unpack("<I", raw[pos + 4:pos + 8])[0]
        body = raw[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            fmt = struct.unpack("<HHIIHH", body[:16])
        elif cid == b"data":
            data = body
        pos += 8 + size + (size & 1)
    if fmt is None or data is None:
        raise ValueError("missing fmt or data chunk")
    tag, channels, rate, _, _, bits = fmt
    if tag != 1 or channels != 1 or bits != 16:
        raise ValueError(f"unsupported WAV format tag={tag} channels={channels} bits={bits}")
    return np.frombuffer(data, dtype="<i2").astype(np.int16), rate
