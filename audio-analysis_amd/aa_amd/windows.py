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
                  fmin: float, fmax: float, pad_short_tracks: bool = False, return_span: bool = False):
    """Window views of one track; with ``return_span`` also the track's sample
    range ``(a, b)`` after the short-track widening (the reference's
    ``track_frames = frames[sr_start:sr_end]``, :127-148), which a band-pass
    filter runs over (:152-162)."""
    if freq_start > fmax or freq_end < fmin:  # :116-119, not identified
        return ([], (0, 0)) if return_span else []
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
    if return_span:
        return views, (view.start, view.stop)
    return views


def schedule(n_samples: int, sr: int, tracks: Sequence, segment_length: float, stride: float,
             fmin: float, fmax: float, pad_short_tracks: bool = False, return_spans: bool = False):
    """Window views for every track (objects with start, end, length,
    freq_start, freq_end), in the reference's track order; with
    ``return_spans`` also each track's (a, b) sample range."""
    res = [track_windows(n_samples, sr, t.start, t.end, t.length, t.freq_start, t.freq_end,
                         segment_length, stride, fmin, fmax, pad_short_tracks, return_span=return_spans)
           for t in tracks]
    if return_spans:
        return [r[0] for r in res], [r[1] for r in res]
    return res


def butter_bandpass(lowcut, highcut, fs, order=2):
    """Second-order sections of the reference's Butterworth filter
    (src/identify_tracks.py:1039-1050): band-pass when lowcut > 0, else
    low-pass at highcut."""
    from scipy.signal import butter
    nyq = 0.5 * fs
    btype = "lowpass"
    freqs = []
    if lowcut > 0:
        btype = "bandpass"
        freqs.append(lowcut / nyq)
    freqs.append(highcut / nyq)
    return butter(order, freqs, analog=False, btype=btype, output="sos")


def filtered_sources(frames: np.ndarray, sr: int, tracks: Sequence, views: List[List[WindowView]],
                     spans, filter_freqs: bool, filter_below, base: int):
    """Band-pass filtered track buffers (src/identify_tracks.py:152-162).

    A track is filtered when the model group's ``filter_freq`` is set, or when
    ``filter_below`` is set and the track's ``freq_end`` is below it; the
    reference then runs ``sosfilt`` over the track's whole sample range once
    (zero initial state at the range start) and cuts its windows from the
    filtered copy.  This host step (scipy's own sosfilt, as the reference; a
    per-track sequential IIR) produces that copy; the windows are remapped to
    it so the device front end reads filtered samples.  Returns (float32 buffer
    of all filtered copies to append after ``base`` samples of PCM, remapped
    views)."""
    from scipy.signal import sosfilt
    pieces, out = [], []
    off = base
    for t, tv, (a, b) in zip(tracks, views, spans):
        if tv and (filter_freqs or (filter_below and t.freq_end < filter_below)):
            y = sosfilt(butter_bandpass(t.freq_start, t.freq_end, sr), frames[a:b]).astype(np.float32)
            pieces.append(y)
            out.append([(off + (src - a), n, p) if n else (src, n, p) for (src, n, p) in tv])
            off += len(y)
        else:
            out.append(tv)
    extra = np.concatenate(pieces) if pieces else np.zeros(0, np.float32)
    return extra, out
