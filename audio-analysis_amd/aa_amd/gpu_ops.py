"""Small device helpers around libaa.so used by the classify() host code."""
from __future__ import annotations

from functools import lru_cache

import numpy as np
import torch

from . import _lib


def _dev(device):
    return torch.device(device or "cuda")


def get_end_spans(n_samples: int, sr: int):
    """Chunks of the reference's get_end scan (src/identify_tracks.py:387-413)
    as sample spans: chunk c covers frames [170 c, 170 c + 170) of a centred
    STFT with n_fft = sr // 10, hop 281, i.e. samples
    [f0 * 281 - n_fft/2, f1 * 281 + n_fft/2) clipped to the recording.
    Memoised per (length, rate): a corpus repeats a few recording lengths
    (callers offset a copy of the span array; the cached one is read-only)."""
    return _get_end_spans(int(n_samples), int(sr))


@lru_cache(maxsize=256)
def _get_end_spans(n_samples: int, sr: int):
    hop = 281
    n_fft = sr // 10
    chunk = sr // hop
    n_frames = 1 + n_samples // hop
    spans, starts = [], []
    start, end = 0, chunk
    while end < n_frames:
        a = max(start * hop - n_fft // 2, 0)
        b = min((end - 1) * hop + n_fft // 2 + (n_fft % 2), n_samples)
        spans.append((a, max(a, b)))
        starts.append(start)
        start, end = end, end + chunk
    arr = np.asarray(spans, dtype=np.int64).reshape(-1, 2)
    arr.flags.writeable = False
    return arr, tuple(starts), hop


def get_end(frames, sr, device=None, pcm_dev=None):
    n = len(frames)
    spans, starts, hop = get_end_spans(n, sr)
    if len(starts) == 0:
        return n / sr
    dev = _dev(device)
    pcm = pcm_dev if pcm_dev is not None else torch.from_numpy(np.ascontiguousarray(frames, np.float32)).to(dev)
    sp = torch.from_numpy(np.array(spans)).to(dev)
    flags = torch.empty(len(starts), dtype=torch.int32, device=dev)
    _lib.check(_lib.lib().aa_span_nonzero(_lib.dptr(pcm), n, _lib.dptr(sp), len(starts), _lib.dptr(flags),
                                          _lib.stream_ptr()), "aa_span_nonzero")
    f = flags.cpu().numpy()
    zero = np.flatnonzero(f == 0)
    if len(zero) == 0:
        return n / sr
    return starts[zero[0]] * hop // sr
