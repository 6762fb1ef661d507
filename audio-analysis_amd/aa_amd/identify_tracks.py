"""``classify()`` and its result types on the MI355X path.

Surface kept from the reference (src/identify_tracks.py):
  classify(file, models, analyse_tracks, meta_data=None)
      -> (tracks, length, signals, raw_length, bird_labels)        :416-573
  Signal (:915-1033), ModelResult (:869-912), Prediction (:845-866),
  get_master_tag (:580-647), load_recording (:49-62), get_end (:387-413),
  signal_noise (:650-706), merge_signals / get_tracks_from_signals (:725-842),
  segment_overlap / mel_freq (:709-718), NON_BIRD / DEFAULT_* constants.

What runs where: decode on the host; the window schedule on the host
(integers only, aa_amd.windows); log-mel front end, CNN ensemble, per-track
mean, the end-of-recording scan and the signal detector on the GPU through
libaa.so; the track builder (merging a few dozen signals) on the host.  The JSON-facing
objects below are plain host bookkeeping, identical in content to the
reference's.
"""
from __future__ import annotations

import logging
from pathlib import Path

import numpy as np

CALL_LENGTH = 1
DEFAULT_SPECIES = ["kiwi", "whistler", "morepork"]
NON_BIRD = ["human", "noise", "insect"]
SPECIFIC_NOISE = ["insect"]
DEFAULT_BIRDS = ["bird"] + DEFAULT_SPECIES
SIGNAL_WIDTH = 0.25
MAX_FRQUENCY = 48000 / 2


def get_max_chirps(length):
    return int(length / (SIGNAL_WIDTH + 0.01))


def segment_overlap(first, second):
    """Length of the intersection of two [start, end] spans (negative = gap)."""
    return (first[1] - first[0]) + (second[1] - second[0]) - (
        max(first[1], second[1]) - min(first[0], second[0]))


_MEL = {}


def mel_freq(f):
    """2595 log10(1 + f / 700) (:712-713), memoised per frequency: the
    detector's signals take their frequencies from the 2049 STFT bins, and
    numpy's scalar arithmetic costs ~8 us a call -- the same value each time."""
    m = _MEL.get(f)
    if m is None:
        m = 2595.0 * np.log10(1.0 + f / 700.0)
        if len(_MEL) < (1 << 16):
            _MEL[f] = m
    return m


# ---------------------------------------------------------------------------
# result types (JSON content identical to the reference's get_meta)
# ---------------------------------------------------------------------------
class Prediction:
    def __init__(self, what, confidence, ebird_id, threshold_used=None, normalize_confidence=True):
        self.what = what
        # banker's rounding of the float32 score x 100, like round(100 * p)
        self.confidence = round(100 * confidence) if normalize_confidence else confidence
        self.ebird_id = ebird_id
        self.filtered = False
        self.threshold_used = threshold_used

    def get_meta(self):
        return {
            "label": self.what,
            "confidence": self.confidence,
            "filtered": self.filtered,
            "ebird_id": self.ebird_id,
            "threshold_used": self.threshold_used,
        }


class ModelResult:
    def __init__(self, model, pre_model):
        self.model = model
        self.pre_model = pre_model
        self.raw_prediction = None
        self.predictions = []

    def add_prediction(self, what, confidence, ebird_ids, threshold_used, normalize_confidence=True):
        eid = None if (ebird_ids is not None and len(ebird_ids) == 0) else ebird_ids
        self.predictions.append(Prediction(what, confidence, eid, threshold_used, normalize_confidence))

    def get_meta(self):
        meta = {"model": self.model, "pre_model": self.pre_model,
                "predictions": [p.get_meta() for p in self.predictions]}
        if self.raw_prediction is not None:
            meta["raw_prediction"] = self.raw_prediction.get_meta()
        return meta


class Signal:
    def __init__(self, start, end, freq_start, freq_end):
        self._set(start, end, freq_start, freq_end, mel_freq(freq_start), mel_freq(freq_end))

    @classmethod
    def _with_mel(cls, start, end, freq_start, freq_end, mel_start, mel_end):
        """A Signal whose mel values are already known (the native track
        builder returns them with the frequencies they belong to)."""
        s = cls.__new__(cls)
        s._set(start, end, freq_start, freq_end, mel_start, mel_end)
        return s

    def _set(self, start, end, freq_start, freq_end, mel_start, mel_end):
        self.start = start
        self.end = end
        self.freq_start = freq_start
        self.freq_end = freq_end
        self.mel_freq_start = mel_start
        self.mel_freq_end = mel_end
        self.results = []
        self.master_tag = None
        self.master_model = None
        self.master_below_thresh = True
        self.track_id = None

    # geometry
    @property
    def length(self):
        return self.end - self.start

    @property
    def freq_range(self):
        return self.freq_end - self.freq_start

    @property
    def mel_freq_range(self):
        return self.mel_freq_end - self.mel_freq_start

    def time_overlap(self, other):
        return segment_overlap((self.start, self.end), (other.start, other.end))

    def mel_freq_overlap(self, other):
        return segment_overlap((self.mel_freq_start, self.mel_freq_end),
                               (other.mel_freq_start, other.mel_freq_end))

    def freq_overlap(self, other):
        return segment_overlap((self.freq_start, self.freq_end), (other.freq_start, other.freq_end))

    def copy(self):
        return Signal(self.start, self.end, self.freq_start, self.freq_end)

    def _refresh_mel(self):
        self.mel_freq_start = mel_freq(self.freq_start)
        self.mel_freq_end = mel_freq(self.freq_end)

    def enlarge(self, scale, min_track_length):
        grown = max(self.length * scale, min_track_length)
        pad = (grown - self.length) / 2
        self.start = max(self.start - pad, 0)
        self.end = self.end + pad
        fpad = ((self.freq_end - self.freq_start) * scale - (self.freq_end - self.freq_start)) / 2
        lo = self.freq_start - fpad
        self.freq_end = int(self.freq_end + fpad)
        self.freq_start = int(max(lo, 0))
        self._refresh_mel()

    def merge(self, other):
        self.start = min(self.start, other.start)
        self.end = max(self.end, other.end)
        self.freq_start = min(self.freq_start, other.freq_start)
        self.freq_end = max(self.freq_end, other.freq_end)
        self._refresh_mel()

    def to_array(self, decimals=1):
        a = [self.start, self.end, self.freq_start, self.freq_end]
        return a if decimals is None else list(np.round(np.array(a), decimals))

    def set_master_tag(self):
        tag = get_master_tag(self)
        if tag is None:
            return
        self.master_tag, self.master_model, self.master_below_thresh = tag

    def get_meta(self):
        meta = {"begin_s": self.start, "end_s": self.end, "freq_start": self.freq_start,
                "freq_end": self.freq_end}
        if self.master_tag is not None:
            meta["master_tag"] = {"below_thresh": self.master_below_thresh,
                                  "prediction": self.master_tag.get_meta(),
                                  "model": self.master_model}
        meta["model_results"] = [r.get_meta() for r in self.results]
        if self.track_id is not None:
            meta["track_id"] = self.track_id
        return meta

    def __str__(self):
        return f"Signal: {self.start}-{self.end} f: {self.freq_start}-{self.freq_end}"


def get_master_tag(track):
    """Pick the track's master tag (src/identify_tracks.py:580-647): the most
    confident specific (non-"bird") unfiltered prediction of the main models,
    unless the pre-model says noise/human over a morepork; else the pre-model's
    first prediction; else the best raw (below-threshold) prediction."""
    pre = None
    sure, raws = [], []
    for r in track.results:
        if r.pre_model:
            pre = r
            continue
        sure.extend((p, r.model) for p in r.predictions if not p.filtered)
        if r.raw_prediction is not None:
            raws.append((r.raw_prediction, r.model))
    best = None
    if sure:
        ranked = sorted(sure, key=lambda pm: pm[0].confidence, reverse=True)
        best = next((pm for pm in ranked if pm[0].what != "bird"), ranked[0])
    pre_pick = None
    if pre is not None and pre.predictions and not pre.predictions[0].filtered:
        pre_pick = (pre.predictions[0], pre.model)
    if best is None and pre_pick is not None:
        return (*pre_pick, False)
    if best is not None:
        if pre_pick is not None and best[0].what == "morepork" and pre_pick[0].what in ("human", "noise"):
            return (*pre_pick, False)
        return (*best, False)
    if raws:
        return (*sorted(raws, key=lambda pm: pm[0].confidence, reverse=True)[0], True)
    if pre is not None and pre.raw_prediction is not None:
        return pre.raw_prediction, pre.model, True
    return None


# ---------------------------------------------------------------------------
# decode (host) and the end-of-recording scan (GPU)
# ---------------------------------------------------------------------------
# decoded recordings handed over by a prefetching caller (aa_amd.corpus):
# {(str(path), resample): (frames, sr)}, each entry consumed once
_PREFETCHED = {}


def load_recording(file, resample=48000):
    from .audio import decode
    hit = _PREFETCHED.pop((str(file), resample), None)
    if hit is not None:
        return hit
    try:
        frames, sr = decode(file)
        if resample is not None and resample != sr:
            from .audio import resample as resample_to
            frames = resample_to(frames, sr, resample)  # librosa.resample (soxr_hq), on the GPU
            sr = resample
        return frames, sr
    except Exception:
        logging.error("Could not load %s", file, exc_info=True)
        raise Exception(f"Could not load {file}")


def get_end(frames, sr, device=None, pcm_dev=None):
    """Reference get_end (:387-413): the start (whole seconds) of the first
    170-frame chunk of the 4800/281 STFT whose 120-band mel block is constant,
    else the recording length.  A block is constant exactly when every frame
    in it sees only zero samples (any nonzero sample gives a nonzero windowed
    spectrum), so the GPU scans sample spans for nonzero values instead of
    computing the STFT."""
    from . import gpu_ops
    return gpu_ops.get_end(frames, sr, device=device, pcm_dev=pcm_dev)


# ---------------------------------------------------------------------------
# signals and the track builder
# ---------------------------------------------------------------------------
def signal_noise(frames, sr, hop_length=281, device=None, pcm_dev=None):
    """Reference signal_noise (:650-706): the recording's spectral blobs as
    Signals, computed on the GPU (aa_amd.signals / aa_signal.hip)."""
    from .signals import detector
    det = detector(sr, hop_length, device)
    return [Signal(*t) for t in det.signal_noise(frames, pcm=pcm_dev)]


def merge_signals(signals):
    """One merge sweep (:725-792): signals sorted by start (ties: higher
    mel_freq_end first); each absorbs the first other signal on the same side
    of 1500 mel that overlaps it enough in time and mel frequency, or lies
    within 2 s with a similar mel range.  Absorbed signals are dropped."""
    to_delete = []
    something_merged = False
    signals = sorted(signals, key=lambda s: s.mel_freq_end, reverse=True)
    signals = sorted(signals, key=lambda s: s.start)
    for s in signals:
        if s in to_delete:
            continue
        merged = False
        for u in signals:
            if u in to_delete or u == s:
                continue
            same_side = (u.mel_freq_end < 1500 and s.mel_freq_end < 1500) or (
                u.mel_freq_end > 1500 and s.mel_freq_end > 1500)
            if not same_side:
                continue
            overlap = s.time_overlap(u)
            freq_overlap_time = 0.5 if (s.mel_freq_start > 1000 and u.mel_freq_start > 1000) else 0.75
            time_diff = s.start - u.end if s.start > u.end else u.start - s.end
            mel_overlap = s.mel_freq_overlap(u)
            if overlap > u.length * 0.75 and mel_overlap > -20:
                s.merge(u)
                merged = True
                break
            elif overlap > 0 and mel_overlap > u.mel_freq_range * freq_overlap_time:
                s.merge(u)
                merged = True
                break
            elif mel_overlap > u.mel_freq_range * freq_overlap_time and time_diff <= 2:
                # (sic) the reference compares u's mel end with s's mel range
                if u.mel_freq_end > s.mel_freq_range:
                    range_overlap = s.mel_freq_range / u.mel_freq_range
                else:
                    range_overlap = u.mel_freq_range / s.mel_freq_range
                if range_overlap < 0.75:
                    continue
                s.merge(u)
                merged = True
                break
        if merged:
            something_merged = True
            to_delete.append(u)
    for s in to_delete:
        signals.remove(s)
    return signals, something_merged


def get_tracks_from_signals(signals, end):
    """Tracks from signals (:795-842): merge until stable, drop signals
    shorter than the running ``min_length`` (0.35 s, then rebound by the
    overlap test as in the reference), enlarge by 1.4 (at least 0.7 s, clipped
    to ``end``), absorb signals overlapping > 70 % of the shorter one, drop
    tracks narrower than 50 mel."""
    merged = True
    while merged:
        signals, merged = merge_signals(signals)
    to_delete = []
    min_length = 0.35
    min_track_length = 0.7
    for s in signals:
        if s in to_delete:
            continue
        if s.length < min_length:
            to_delete.append(s)
            continue
        s.enlarge(1.4, min_track_length=min_track_length)
        s.end = min(end, s.end)
        for s2 in signals:
            if s2 in to_delete or s == s2:
                continue
            overlap = s.time_overlap(s2)
            min_length = min(s.length, s2.length)
            if overlap > 0.7 * min_length:
                s.merge(s2)
                to_delete.append(s2)
    for s in to_delete:
        signals.remove(s)
    narrow = [s for s in signals if s.mel_freq_range < 50]
    for s in narrow:
        signals.remove(s)
    return signals


_MEL_INT = None
_MEL_INT_PTR = 0


def _mel_int_table():
    """mel_freq of the integer frequencies 0 .. 2^17 - 1 (enlarge's int()
    results) in one numpy evaluation, for aa_tracks_from_signals; checked
    against mel_freq's scalar path on every 64th entry (numpy's log10 is its
    own, not libm's; its array and scalar paths agree -- where they would
    not, False: the Python builder runs)."""
    global _MEL_INT, _MEL_INT_PTR
    if _MEL_INT is None:
        t = 2595.0 * np.log10(1.0 + np.arange(1 << 17, dtype=np.float64) / 700.0)
        ok = all(t[f] == 2595.0 * np.log10(1.0 + f / 700.0) for f in range(0, 1 << 17, 64))
        _MEL_INT = t if ok else False
        _MEL_INT_PTR = t.ctypes.data if ok else 0
    return _MEL_INT


def _is_int(v):
    t = type(v)
    if t is float or t is np.float64:
        return 0
    return int(t is int or (isinstance(v, (int, np.integer)) and t is not bool))


def tracks_from_signals(signals, end):
    """get_tracks_from_signals (:795-842) of copies of ``signals`` (they are
    left as they are), through libaa's host builder aa_tracks_from_signals
    (csrc/aa_tracks.cpp: the same double arithmetic, ints kept ints): the same
    tracks, field for field and type for type.  Python's own builder runs
    where the native one declines (a zero mel range, where Python raises; a
    frequency past the mel table)."""
    import ctypes as C
    from . import _lib
    n = len(signals)
    lut = _mel_int_table()
    if n == 0 or lut is False:
        return get_tracks_from_signals([s.copy() for s in signals], end)
    # one f64 buffer: n input rows, then n output rows; one i32 buffer: n
    # input kinds, then n output kinds
    buf = np.empty((2 * n, 6), dtype=np.float64)
    buf[:n] = [(s.start, s.end, s.freq_start, s.freq_end, s.mel_freq_start, s.mel_freq_end) for s in signals]
    kind = np.empty(2 * n, dtype=np.int32)
    kind[:n] = [_is_int(s.start) | _is_int(s.end) << 1 | _is_int(s.freq_start) << 2 | _is_int(s.freq_end) << 3
                for s in signals]
    b, k = buf.ctypes.data, kind.ctypes.data
    m = C.c_int64(0)
    rc = _lib.lib().aa_tracks_from_signals(b, k, n, float(end), _is_int(end), _MEL_INT_PTR, lut.size,
                                           b + 48 * n, k + 4 * n, C.byref(m))
    if rc in (_lib.AA_ERR_INVALID, _lib.AA_ERR_UNSUPPORTED):
        return get_tracks_from_signals([s.copy() for s in signals], end)
    _lib.check(rc, "aa_tracks_from_signals")
    m = m.value
    return [Signal._with_mel(int(r[0]) if f & 1 else r[0], int(r[1]) if f & 2 else r[1],
                             int(r[2]) if f & 4 else r[2], int(r[3]) if f & 8 else r[3], r[4], r[5])
            for r, f in zip(buf[n:n + m].tolist(), kind[n:n + m].tolist())]


# ---------------------------------------------------------------------------
# classify
# ---------------------------------------------------------------------------
def _group_models(models):
    from .model import load_model_meta
    pre, main = [], []
    for m in models:
        meta = load_model_meta(Path(m))
        (pre if meta.get("pre_model", False) else main).append((m, meta))
    groups = [main]
    if pre:
        groups.append(pre)
    return groups


def classify(file, models, analyse_tracks, meta_data=None, precision=None, device=None):
    """Reference classify (:416-573): decode, get_end, signal_noise on every
    recording; tracks from the metadata (analyse_tracks) or built from the
    signals; the model groups over every track's windows."""
    import torch
    from .pipeline import Classifier
    frames, sr = load_recording(file)
    raw_length = len(frames) / sr
    dev = torch.device(device or "cuda")
    pcm = torch.from_numpy(np.ascontiguousarray(frames, dtype=np.float32)).to(dev)  # uploaded once
    length = get_end(frames, sr, device=dev, pcm_dev=pcm)
    n_sig = int(sr * length)
    signals = signal_noise(frames[:n_sig], sr, 281, device=dev, pcm_dev=pcm[:n_sig])
    if analyse_tracks:
        if meta_data is None:
            return None
        tracks = []
        for t in meta_data["Tracks"]:
            s = Signal(t["start"], t["end"], t.get("minFreq", 0), t.get("maxFreq", MAX_FRQUENCY))
            s.track_id = t["id"]
            tracks.append(s)
    else:
        tracks = tracks_from_signals(signals, length)
    if len(tracks) == 0:
        return [], length, [], raw_length, []
    clf = Classifier.shared(precision=precision, device=dev)
    bird_labels = clf.classify_tracks(frames, sr, tracks, _group_models(models), pcm=pcm)
    if bird_labels is None:
        return [], length, [], raw_length, []
    return tracks, length, signals, raw_length, list(bird_labels)
