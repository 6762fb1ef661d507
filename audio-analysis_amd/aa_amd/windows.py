"""Sliding-window scheduler: which samples of a recording form each window.

The reference (src/identify_tracks.py:65-199, ``load_samples``) slices numpy
arrays inside its per-window loop.  Here the same decisions are made once on
the host and emitted as integer window views ``(src, n_valid, pad_left)``
(struct aa_window, include/aa.h) for the GPU front end; no samples are copied.
Python slicing semantics are reproduced exactly by slicing ``range`` objects,
and ``np.random.randint`` is drawn in the reference's order (short track
placement :132, short window padding :167), so a seeded global RandomState gives
the reference's windows bit-for-bit (tests/golden/windows.json).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

WindowView = Tuple[int, int, int]  # (src, n_valid, pad_left)


def track_windows(n_samples: int, sr: int, start: float, end: float, length: float,
                  freq_start: float, freq_end: float, segment_length: float, stride: float,
                  fmin: float, fmax: float, pad_short_tracks: bool = False) -> List[WindowView]:
    if freq_start > fmax or freq_end < fmin:  # :116-119, not identified
        return []
    size = int(sr * segment_length)
    a = int(sr * start)
    b = int(end * sr)
    if not pad_short_tracks:
        short = size - (b - a)
        if short > 0:  # :130-146, widen to one full window at a random offset
            off = np.random.randint(0, short)
            a -= off
            if a <= 0:
                a = 0
                b = min(size, n_samples)
            else:
                stop = b + short - off
                if stop > n_samples:
                    stop = n_samples
                    a = max(stop - size, 0)
                b = stop
            if b - a != size:
                raise AssertionError("recording shorter than one segment")  # :146
    view = range(n_samples)[a:b]
    views: List[WindowView] = []
    t = 0.0
    lo, hi = 0, min(b, size)
    while True:
        sub = view[lo:hi]
        n_valid = len(sub)
        src = sub.start if n_valid else 0
        pad_left = 0
        if n_valid != size:  # :165-168
            pad_left = int(np.random.randint(0, size - n_valid))
        views.append((int(src), int(n_valid), pad_left))
        t += stride
        seg_end = t + segment_length
        lo = int(t * sr)
        hi = min(int(seg_end * sr), lo + size)
        if seg_end > length:  # at least one window, stop past the track end
            break
    return views


def schedule(n_samples: int, sr: int, tracks: Sequence, segment_length: float, stride: float,
             fmin: float, fmax: float, pad_short_tracks: bool = False) -> List[List[WindowView]]:
    """Window views for every track (objects with start, end, length,
    freq_start, freq_end), in the reference's track order."""
    return [track_windows(n_samples, sr, t.start, t.end, t.length, t.freq_start, t.freq_end,
                          segment_length, stride, fmin, fmax, pad_short_tracks) for t in tracks]
