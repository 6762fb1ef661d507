"""Device orchestration of one recording's classification.

Mirrors the model-group loop of the reference classify()
(src/identify_tracks.py:444-571): models split into the mean ensemble and
the pre-model group; the FIRST model of the first group configures the front
end and the windows are computed once and reused by later groups (:501-529);
per group: every model predicts every window, np.mean over models then over
each track's windows, threshold -> Prediction / raw_prediction.

MI355X shape of the same work: the recording is uploaded once; all windows of
all tracks form one batch (window views are integers, no sample copies); one
aa_fe_run for the batch, one aa_model_forward per model, one aa_track_mean
per group, then a single device->host copy of [n_tracks, n_labels] scores.
Models and front-end plans are cached across recordings.
"""
from __future__ import annotations

import dataclasses
import logging
import os
import threading
from pathlib import Path

import numpy as np
import torch

from .frontend import FeSettings, FrontEnd, pack_windows
from .model import Model, track_mean
from .windows import filtered_sources, schedule


def fe_settings_from_meta(meta: dict, sr: int) -> FeSettings:
    """Front-end keys with the reference's defaults (:466-497)."""
    n_fft = meta.get("n_fft", 4096)
    return FeSettings(
        sr=sr,
        segment_length=meta.get("segment_length", 3),
        n_fft=4096 if n_fft is None else n_fft,
        hop_length=meta.get("hop_length", 640),
        n_mels=meta.get("n_mels", 160),
        fmin=meta.get("fmin", 50),
        fmax=meta.get("fmax", 11000),
        break_freq=meta.get("break_freq", 1750),
        htk=meta.get("htk", False),
        power=meta.get("power", 2),
        db_scale=meta.get("db_scale", True),
        normalize=meta.get("normalize", True),
        mean_sub=meta.get("mean_sub", False),
        channels=meta.get("channels", 1),
    )


class Classifier:
    _shared = {}

    @classmethod
    def shared(cls, precision=None, device=None):
        precision = precision or os.environ.get("AA_PRECISION", "bf16x3")
        key = (precision, str(device or "cuda"))
        if key not in cls._shared:
            cls._shared[key] = cls(precision, device)
        return cls._shared[key]

    def __init__(self, precision="bf16x3", device=None):
        self.precision = precision
        self.device = torch.device(device or "cuda")
        self._models = {}
        self._fes = {}
        self._lock = threading.RLock()
        self.windows_done = 0  # windows through the front end (bench.py's configs[3] roofline)

    def frontend(self, s: FeSettings) -> FrontEnd:
        with self._lock:
            if s not in self._fes:
                self._fes[s] = FrontEnd(s, self.device)
            return self._fes[s]

    def model(self, path, meta, in_shape) -> Model:
        key = (str(Path(path).resolve()), tuple(in_shape))
        with self._lock:
            if key not in self._models:
                logging.info("Loading %s", str(path))
                self._models[key] = Model(path, in_shape, precision=self.precision, device=self.device,
                                          meta=meta)
            return self._models[key]

    def classify_tracks(self, frames, sr, tracks, groups, pcm=None):
        """One recording (classify()): the batch core below with one entry,
        the caller's RandomState as it is."""
        dev = self.device
        if pcm is None:
            pcm = torch.from_numpy(np.ascontiguousarray(frames, dtype=np.float32)).to(dev)
        rec = BatchRec(n=len(frames), off=0, tracks=tracks, frames=lambda: frames, seed=None)
        res = self.classify_batch(pcm, sr, [rec], groups, raise_errors=True)[0]
        if isinstance(res, BaseException):
            raise res
        return res

    def classify_batch(self, pcm, sr, recs, groups, raise_errors=False, ws=None):
        """The model-group loop of classify() (src/identify_tracks.py:444-571)
        for several recordings at once: every recording's windows in one
        front-end launch set, one forward per model, one track mean, one
        device->host copy.  ``pcm``: device f32 holding recording r at
        ``recs[r].off``.  A recording with ``seed`` set reseeds numpy's global
        RandomState right before its window schedule (what aa_amd.corpus does
        per file), so its windows do not depend on its batch neighbours.
        Returns per recording the bird labels (a set), or the exception the
        single-recording path would have raised for it (non-finite audio);
        the results land on each recording's tracks.  ``raise_errors``: raise
        a recording's exception instead (the single-recording path).  ``ws``:
        a dict of this caller's device workspaces (grown here), for callers
        that run several batches concurrently on their own streams."""
        from .identify_tracks import DEFAULT_BIRDS
        dev = self.device
        R = len(recs)
        errs = [None] * R
        views = None  # per recording: per track window views (global sample offsets)
        logmel = rows = fe = None
        status_host = status_views = None
        bird_labels = set()
        for group in groups:
            if len(group) > 1:
                logging.info("Meaning predictions as have multiple models")
            meta = group[0][1]  # IndexError on an empty group, as the reference
            s = fe_settings_from_meta(meta, sr)
            if meta.get("use_mfcc", False):
                # get_spect's MFCC branch (:269-280): librosa.feature.mfcc + tf.image.resize_with_pad
                raise NotImplementedError("MFCC features (use_mfcc)")
            labels = meta.get("labels")
            model_name = meta.get("name", False)
            bird_labels.update(meta.get("bird_labels", DEFAULT_BIRDS))
            if model_name == "embeddings":
                raise NotImplementedError("tensorflow_hub embedding models need a network fetch")
            if views is None:
                views, extras = [], []
                extra_at = int(pcm.numel())
                for i, r in enumerate(recs):
                    try:
                        if r.seed is not None:
                            with _RNG_LOCK:  # numpy's global RandomState: seed and draws together
                                np.random.seed(r.seed)
                                v, spans = schedule(r.n, sr, r.tracks, s.segment_length,
                                                    meta.get("segment_stride", 1.5), s.fmin, s.fmax,
                                                    meta.get("pad_short_tracks", False), return_spans=True)
                        else:
                            v, spans = schedule(r.n, sr, r.tracks, s.segment_length, meta.get("segment_stride", 1.5),
                                                s.fmin, s.fmax, meta.get("pad_short_tracks", False), return_spans=True)
                        # band-pass filtered tracks (:152-162): their windows read a
                        # filtered copy appended after the batch's samples
                        ff, fb = meta.get("filter_freq", False), meta.get("filter_below", None)
                        if ff or fb:
                            extra, v = filtered_sources(r.frames(), sr, r.tracks, v, spans, ff, fb, extra_at - r.off)
                            if len(extra):
                                extras.append(extra)
                                extra_at += len(extra)
                    except Exception as e:
                        if raise_errors:
                            raise
                        errs[i] = e  # (e.g. :146's assertion on a recording shorter than a window)
                        v = [[] for _ in r.tracks]
                    views.append([[(src + r.off, n, p) for (src, n, p) in tv] for tv in v])
                if extras:
                    pcm = torch.cat([pcm, torch.from_numpy(np.concatenate(extras)).to(dev)])
                flat = [w for rv in views for tv in rv for w in tv]
                fe = self.frontend(s)
                if flat:
                    rows = torch.from_numpy(pack_windows(flat, int(pcm.numel()), win_len=s.win_len)).to(dev)
                    status = torch.empty(len(flat), dtype=torch.int32, device=dev)
                    logmel = fe.run(pcm, rows, status=status, workspace=_grow(ws, "fe", fe.workspace_bytes(len(flat)), dev))
                    # per-window status, read back with the first group's scores
                    # (one host sync per batch, not two)
                    status_host = torch.empty(len(flat), dtype=torch.int32, pin_memory=True)
                    status_host.copy_(status, non_blocking=True)
                    status_views = views
            else:
                logging.info("Re using track data this will cuase problems if the STFT settings are "
                             "not the same for multiple models")
            counts = [[len(tv) for tv in rv] for rv in views]
            total = sum(sum(c) for c in counts)
            if total == 0:
                continue
            if group is groups[0]:
                with self._lock:
                    self.windows_done += total
            group_mel = logmel
            if "efficientnet" in model_name.lower():
                # np.repeat(d, 3, -1) of the shared windows (:539-540): every
                # channel is the same log-mel, so this is the first group's
                # front end with three times the channels
                fe3 = self.frontend(dataclasses.replace(fe.s, channels=fe.s.channels * 3))
                group_mel = fe3.run(pcm, rows, workspace=_grow(ws, "fe", fe3.workspace_bytes(int(rows.shape[0])), dev))
            probs = torch.empty((len(group), total, len(labels)), dtype=torch.float32, device=dev)
            for k, (path, m_meta) in enumerate(group):
                m = self.model(path, m_meta, group_mel.shape[1:])
                if m.n_labels != len(labels):
                    raise ValueError(f"{path}: {m.n_labels} outputs for {len(labels)} labels")
                m.forward(group_mel, probs=probs[k], workspace=_grow(ws, "model", m.workspace_bytes(total), dev))
            # one track mean over every recording's tracks that have windows
            flat_counts = np.asarray([c for rc in counts for c in rc], np.int64)
            begin = np.concatenate([[0], np.cumsum(flat_counts)[:-1]]).astype(np.int32)
            sel = np.flatnonzero(flat_counts > 0)
            wb = torch.from_numpy(begin[sel]).to(dev)
            wc = torch.from_numpy(flat_counts[sel].astype(np.int32)).to(dev)
            means = track_mean(probs, wb, wc).cpu().numpy()
            if status_host is not None:  # ready: the copy preceded the means on the stream
                st = status_host.numpy()
                status_host = None
                if st.any():  # librosa valid_audio, per recording
                    k = 0
                    for i, rv in enumerate(status_views):
                        nw = sum(len(tv) for tv in rv)
                        if st[k:k + nw].any():
                            errs[i] = ValueError("Audio buffer is not finite everywhere")
                        k += nw
            row, t0 = 0, 0
            for i, (r, rc) in enumerate(zip(recs, counts)):
                nt = len(rc)
                mine = [t for t in range(nt) if rc[t] > 0]
                if mine and errs[i] is None:  # (a recording with no windows skips the group, :530-531)
                    apply_group_scores(r.tracks, mine, means[row:row + len(mine)], meta)
                row += len(mine)
                t0 += nt
        return [e if e is not None else set(bird_labels) for e in errs]


_RNG_LOCK = threading.Lock()


def _grow(ws, key, need, dev):
    """A caller-owned workspace (None: the plan's own)."""
    if ws is None:
        return None
    t = ws.get(key)
    if t is None or t.numel() < need:
        t = ws[key] = torch.empty(max(int(need), 256), dtype=torch.uint8, device=dev)
    return t


@dataclasses.dataclass
class BatchRec:
    """One recording of a classify_batch call."""
    n: int                 # samples
    off: int               # first sample in the batch's device PCM
    tracks: list           # Signal objects; results are appended to them
    frames: object         # callable -> host float32 samples (band-pass filtering only)
    seed: object = None    # np.random.seed before this recording's window schedule


def apply_group_scores(tracks, track_idx, means, meta):
    """Per-track mean scores of one model group -> ModelResult (reference
    src/identify_tracks.py:552-571): labels with p >= threshold become
    Predictions (confidence = round(100 p)); with none, the arg-max becomes
    the raw_prediction.  ``means`` rows are float32 like numpy's mean."""
    from .identify_tracks import ModelResult, Prediction
    labels = meta.get("labels")
    ebird_ids = meta.get("ebird_ids")
    thr = meta.get("threshold", 0.7)
    for row, ti in enumerate(track_idx):
        prediction = means[row]
        result = ModelResult(meta.get("name", False), meta.get("pre_model", False))
        tracks[ti].results.append(result)
        best = None
        for i, p in enumerate(prediction):
            if best is None or p > best[1]:
                best = (i, p)
            if p >= thr:
                result.add_prediction(labels[i], p, None if ebird_ids is None else ebird_ids[i], thr)
        if not result.predictions:
            result.raw_prediction = Prediction(labels[best[0]], best[1],
                                               None if ebird_ids is None else ebird_ids[best[0]])
