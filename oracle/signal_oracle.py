"""CPU oracle for signal_noise (the per-recording signal detector).  TEST
INFRASTRUCTURE ONLY: only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it; the product path never does.

What it restates (reference = /root/reference):

* ``signal_noise`` src/identify_tracks.py:650-706
  - ``np.abs(librosa.stft(frames, n_fft=4096, hop_length=281))`` (:654) through
    ``fe_oracle.stft_mag`` (librosa 0.11: centre zero pad, periodic Hann, f64
    rfft stored as complex64, f32 magnitude)
  - normalisation by the global max, row / column medians (numpy's median:
    mean of the two middle values for an even count) and the 3x-median mask
    (:656-669)
  - ``cv2.morphologyEx(MORPH_OPEN, ones(4, 4))``, ``cv2.dilate(ones(h, w))``,
    ``cv2.erode(ones(h // 10, w))`` (:670-684), restated with OpenCV 4.11's
    semantics: anchor at the kernel centre (kw // 2, kh // 2), both erode and
    dilate take ``src(x + i - ax, y + j - ay)`` over the kernel (no reflection),
    out-of-image pixels never change the result (``morphologyDefaultBorderValue``)
    and an empty kernel means a 3x3 rectangle
  - ``cv2.connectedComponentsWithStats`` (8-connectivity) (:686): stats
    ``[left, top, width, height, area]``; the label order of OpenCV's default
    8-connectivity algorithm (Spaghetti, 2x2-block raster scan with min-label
    union-find) is the block-raster order of each component's first 2x2 block,
    which only matters for components that tie on ``left`` in the stable sort
    at :688
  - the size filter and conversion to (start, end, freq_start, freq_end)
    (:689-704)

Parity status: opencv-python 4.11 (requirements.txt) and librosa 0.11 are not
installed and their sources are not under /root/reference, so the
morphology/CCL semantics above are restated from OpenCV's documented
behaviour: "parity unpinned" against cv2 itself.  The GPU implementation is
held bit-exact to this oracle on identical masks, and to its STFT within f32
tolerance.
"""
from __future__ import annotations

import numpy as np

from .fe_oracle import stft_mag

SIGNAL_WIDTH = 0.25  # src/identify_tracks.py:21
N_FFT = 4096


def signal_mask(S: np.ndarray) -> np.ndarray:
    """src/identify_tracks.py:656-669 on a float32 [bins, frames] magnitude."""
    with np.errstate(invalid="ignore", divide="ignore"):
        a_max = np.amax(S)
        S = S / a_max
        row = np.median(S, axis=1)[:, None]
        col = np.median(S, axis=0)[None, :]
        return ((S > 3 * col) & (S > 3 * row)).astype(np.uint8)


def morph(img: np.ndarray, kh: int, kw: int, erode: bool) -> np.ndarray:
    """cv2.erode / cv2.dilate with np.ones((kh, kw)): out[y, x] = min / max of
    img[y + i - kh // 2, x + j - kw // 2] over the kernel, taps outside the
    image ignored.  Separable (a rectangle), so rows then columns."""
    if kh == 0 or kw == 0:  # cv2: empty kernel -> 3x3 rectangle
        kh = kw = 3
    ident = 1 if erode else 0
    red = np.minimum if erode else np.maximum
    H, W = img.shape
    ax, ay = kw // 2, kh // 2
    pad = np.full((H, W + kw - 1), ident, np.uint8)
    pad[:, ax:ax + W] = img
    tmp = np.full((H, W), ident, np.uint8)
    for j in range(kw):
        tmp = red(tmp, pad[:, j:j + W])
    pad = np.full((H + kh - 1, W), ident, np.uint8)
    pad[ay:ay + H] = tmp
    out = np.full((H, W), ident, np.uint8)
    for i in range(kh):
        out = red(out, pad[i:i + H])
    return out


def connected_components_stats(img: np.ndarray) -> np.ndarray:
    """cv2.connectedComponentsWithStats(img)[2][1:] (8-connectivity): int64
    rows [left, top, width, height, area], in OpenCV's label order."""
    from scipy import ndimage

    H, W = img.shape
    lab, n = ndimage.label(img, structure=np.ones((3, 3), dtype=int))
    if n == 0:
        return np.zeros((0, 5), dtype=np.int64)
    ys, xs = np.nonzero(lab)
    ids = lab[ys, xs]
    key = (ys // 2).astype(np.int64) * ((W + 1) // 2) + xs // 2
    first = np.full(n + 1, np.iinfo(np.int64).max, dtype=np.int64)
    np.minimum.at(first, ids, key)
    area = np.bincount(ids, minlength=n + 1)
    rows = []
    for i, sl in enumerate(ndimage.find_objects(lab), start=1):
        rows.append([sl[1].start, sl[0].start, sl[1].stop - sl[1].start, sl[0].stop - sl[0].start,
                     area[i], first[i]])
    rows = np.array(rows, dtype=np.int64)
    rows = rows[np.argsort(rows[:, 5], kind="stable")]
    return rows[:, :5]


def signal_geometry(sr: int, hop_length: int):
    """(width, height, freqs) of src/identify_tracks.py:673-681."""
    width = int(SIGNAL_WIDTH * sr / hop_length)
    freqs = np.fft.rfftfreq(n=N_FFT, d=1.0 / sr)  # librosa.fft_frequencies
    height = 0
    for i, f in enumerate(freqs):
        if f > 100:
            height = i + 1
            break
    return width, height, freqs


def signal_mask_to_stats(sig: np.ndarray, sr: int, hop_length: int) -> np.ndarray:
    """Morphology + components of :670-691: the kept stats rows, sorted."""
    width, height, _ = signal_geometry(sr, hop_length)
    sig = morph(morph(sig, 4, 4, True), 4, 4, False)  # MORPH_OPEN
    sig = morph(sig, height, width, False)
    sig = morph(sig, height // 10, width, True)
    stats = connected_components_stats(sig)
    order = sorted(range(len(stats)), key=lambda i: stats[i][0])
    min_width = 0.65 * width
    min_height = height - height // 10
    return np.array([stats[i] for i in order if stats[i][2] > min_width and stats[i][3] > min_height],
                    dtype=np.int64).reshape(-1, 5)


def stats_to_signals(stats: np.ndarray, sr: int, hop_length: int):
    """(start, end, freq_start, freq_end) tuples of :698-704 (the 281 there is
    literal in the reference)."""
    _, _, freqs = signal_geometry(sr, hop_length)
    out = []
    for s in stats:
        max_freq = min(len(freqs) - 1, int(s[1] + s[3]))
        out.append((int(s[0]) * 281 / sr, (int(s[0]) + int(s[2])) * 281 / sr,
                    freqs[int(s[1])], freqs[max_freq]))
    return out


def signal_noise(frames: np.ndarray, sr: int, hop_length: int = 281):
    """Full restatement of src/identify_tracks.py:650-706 -> (tuples, mask, stats)."""
    S = stft_mag(np.asarray(frames, dtype=np.float32), N_FFT, hop_length)
    sig = signal_mask(S)
    stats = signal_mask_to_stats(sig, sr, hop_length)
    return stats_to_signals(stats, sr, hop_length), sig, stats
