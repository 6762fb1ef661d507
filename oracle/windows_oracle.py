"""CPU oracle for the sliding-window scheduler.  TEST INFRASTRUCTURE ONLY.

Restates ``load_samples`` (src/identify_tracks.py:65-199) with the per-window
spectrogram call replaced by returning the raw window samples, so a test can
compare the product's integer window table (source offset, valid length, left
zero pad) with what the reference would slice.  ``np.random`` is consumed in the
same order as the reference (one ``randint`` per short track at :132, one per
short window at :167), so seeding ``np.random`` reproduces the reference's
random placements.  Pinned against golden window tables captured from the
reference itself (tests/golden/make_golden.py).
"""
from __future__ import annotations

import numpy as np


def track_windows(frames, sr, track, segment_length, stride, fmin, fmax,
                  pad_short_tracks=False):
    """Yield raw (un-normalised) float32 windows for one track, or [] when the
    track lies outside [fmin, fmax] (src/identify_tracks.py:116-119)."""
    if track.freq_start > fmax or track.freq_end < fmin:
        return []
    size = int(sr * segment_length)
    start = 0
    end = start + segment_length
    lo = int(sr * track.start)
    hi = int(track.end * sr)
    if pad_short_tracks:
        end = min(end, track.length)
        seg = frames[lo:hi]
    else:
        missing = size - (hi - lo)
        if missing > 0:
            shift = np.random.randint(0, missing)
            lo = lo - shift
            if lo <= 0:
                lo = 0
                hi = min(lo + size, len(frames))
            else:
                stop = hi + missing - shift
                if stop > len(frames):
                    stop = len(frames)
                    lo = max(stop - size, 0)
                hi = stop
            assert hi - lo == size  # src/identify_tracks.py:146
        seg = frames[lo:hi]
    w_lo = 0
    w_hi = min(hi, size)
    out = []
    while True:
        data = seg[w_lo:w_hi]
        if len(data) != size:
            extra = size - len(data)
            left = np.random.randint(0, extra)
            data = np.pad(data, (left, extra - left))
        out.append(np.asarray(data))
        start = start + stride
        end = start + segment_length
        w_lo = int(start * sr)
        w_hi = min(int(end * sr), w_lo + size)
        if end > track.length:
            break
    return out
