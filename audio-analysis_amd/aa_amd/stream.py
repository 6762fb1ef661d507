"""Streamed classification of many recordings (BASELINE.json configs[2]:
1000 x 60 s clips, model1+model2+model3 sharing one front end).

Reference behaviour per recording: classify() (src/identify_tracks.py:416-573)
runs once per file, the models of a group share the first model's front end
(:465, :501-529), predictions are averaged over models then over each track's
windows (:547-551).  The MI355X shape of the same work: recordings are packed a
few at a time into one batch -- one aa_fe_run over every window of every
track of the batch, one aa_model_forward per ensemble model, one
aa_track_mean -- and PCM reaches the device from pinned host buffers on a copy
stream, double-buffered, so batch i+1's upload overlaps batch i's kernels,
and the two buffer slots compute on their own streams, so batch i+1's
kernels run beside batch i's.
Per-track scores come back in one device->host copy per batch.  Every kernel
works per window / per track, so each recording's scores are bit-identical to
classifying it on its own.
"""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from typing import Iterable, List, Sequence

import numpy as np
import torch

from . import _lib
from .frontend import FeSettings, FrontEnd, pack_windows
from .model import Model
from .windows import schedule


@dataclass
class Recording:
    key: object                 # caller's id, returned with the scores
    pcm: np.ndarray             # float32 mono at the front end's sample rate
    tracks: Sequence = field(default_factory=list)  # objects with start, end, length, freq_start, freq_end


class StreamRunner:
    """Batches recordings through the GPU path with copy/compute overlap.

    ``run`` yields ``(key, track_index, scores)`` per track that has windows,
    in input order; ``scores`` is the float32 [L] mean over models and windows
    (what apply_group_scores thresholds)."""

    def __init__(self, model_paths: Sequence, settings: FeSettings, precision="bf16x3", device=None,
                 max_windows=512, max_samples=16 * 2_880_000, segment_stride=1.5, pad_short_tracks=False,
                 metas=None):
        self.device = torch.device(device or "cuda")
        self.s = settings
        self.fe = FrontEnd(settings, self.device)
        in_shape = self.fe.out_shape(1)[1:]
        metas = metas or [None] * len(model_paths)
        self.models = [Model(p, in_shape, precision=precision, device=self.device, meta=m)
                       for p, m in zip(model_paths, metas)]
        labels = {m.n_labels for m in self.models}
        if len(labels) != 1:
            raise ValueError("ensemble models disagree on the label count")
        self.L = labels.pop()
        self.max_windows, self.max_samples = int(max_windows), int(max_samples)
        self.stride, self.pad_short = segment_stride, pad_short_tracks
        self.copy_stream = torch.cuda.Stream(device=self.device)
        # each slot computes on its own stream: batch i+1's kernels run beside
        # batch i's (the slots own all their buffers), as the bench's
        # two-stream step does
        self.slots = [self._slot() for _ in range(2)]
        self._next = 0
        # host staging copies, one recording per thread (numpy copies run
        # without the GIL): a batch is ~90 MB of PCM, which one core copies
        # more slowly than the GPU classifies it
        self._pool = ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1))

    def _slot(self):
        dev, W, M = self.device, self.max_windows, len(self.models)
        return {
            "h_pcm": torch.empty(self.max_samples, dtype=torch.float32).pin_memory(),
            "d_pcm": torch.empty(self.max_samples, dtype=torch.float32, device=dev),
            "h_win": torch.empty((W, 2), dtype=torch.int64).pin_memory(),
            "d_win": torch.empty((W, 2), dtype=torch.int64, device=dev),
            "h_tr": torch.empty((2, W), dtype=torch.int32).pin_memory(),
            "d_tr": torch.empty((2, W), dtype=torch.int32, device=dev),
            "logmel": torch.empty(self.fe.out_shape(W), dtype=torch.float32, device=dev),
            "logits": torch.empty((M, W, self.L), dtype=torch.float32, device=dev),
            "probs": torch.empty((M, W, self.L), dtype=torch.float32, device=dev),
            "means": torch.empty((W, self.L), dtype=torch.float32, device=dev),
            "h_means": torch.empty((W, self.L), dtype=torch.float32).pin_memory(),
            "fe_ws": torch.empty(max(self.fe.workspace_bytes(W), 256), dtype=torch.uint8, device=dev),
            "m_ws": torch.empty(max(max(m.workspace_bytes(W) for m in self.models), 256), dtype=torch.uint8,
                                device=dev),
            "ks": torch.cuda.Stream(device=dev),
            "uploaded": torch.cuda.Event(),
            "done": torch.cuda.Event(),
            "pending": None,
        }

    def _views(self, rec: Recording):
        s = self.s
        return schedule(len(rec.pcm), s.sr, rec.tracks, s.segment_length, self.stride, s.fmin, s.fmax,
                        self.pad_short)

    def run(self, recordings: Iterable[Recording]):
        batch, n_s, n_w = [], 0, 0
        for rec in recordings:
            views = self._views(rec)
            nw = sum(len(v) for v in views)
            if nw > self.max_windows or len(rec.pcm) > self.max_samples:
                raise ValueError(f"recording {rec.key!r}: {nw} windows / {len(rec.pcm)} samples exceed the "
                                 f"runner's batch ({self.max_windows} / {self.max_samples})")
            if batch and (n_w + nw > self.max_windows or n_s + len(rec.pcm) > self.max_samples):
                yield from self._submit(batch)
                batch, n_s, n_w = [], 0, 0
            batch.append((rec, views))
            n_s += len(rec.pcm)
            n_w += nw
        if batch:
            yield from self._submit(batch)
        for k in range(2):
            yield from self._drain(self.slots[(self._next + k) % 2])

    def _submit(self, batch):
        slot = self.slots[self._next]
        self._next ^= 1
        yield from self._drain(slot)  # its buffers are free once its last batch finished
        # host staging: PCM of the batch back to back, window rows, track ranges
        rows, begins, counts, owners = [], [], [], []
        off = 0
        h_pcm = slot["h_pcm"].numpy()
        copies = []
        for rec, views in batch:
            n = len(rec.pcm)
            copies.append(self._pool.submit(np.copyto, h_pcm[off:off + n], rec.pcm))
            for ti, tv in enumerate(views):
                if not tv:
                    continue
                begins.append(len(rows))
                counts.append(len(tv))
                owners.append((rec.key, ti))
                rows.extend(pack_windows(tv, n, offset=off))
            off += n
        for c in copies:
            c.result()
        nw, nt = len(rows), len(owners)
        if nw:
            slot["h_win"].numpy()[:nw] = np.asarray(rows, dtype=np.int64)
            slot["h_tr"].numpy()[0, :nt] = begins
            slot["h_tr"].numpy()[1, :nt] = counts
        cs, ks = self.copy_stream, slot["ks"]
        # (the slot's previous batch has finished: _drain above synchronised it)
        with torch.cuda.stream(cs):
            slot["d_pcm"][:off].copy_(slot["h_pcm"][:off], non_blocking=True)
            slot["d_win"][:nw].copy_(slot["h_win"][:nw], non_blocking=True)
            slot["d_tr"][:, :nt].copy_(slot["h_tr"][:, :nt], non_blocking=True)
            slot["uploaded"].record(cs)
        ks.wait_event(slot["uploaded"])
        if nw:
            self.fe.run(slot["d_pcm"][:off], slot["d_win"][:nw], out=slot["logmel"][:nw], stream=ks,
                        workspace=slot["fe_ws"])
            for k, m in enumerate(self.models):
                m.forward(slot["logmel"][:nw], slot["logits"][k, :nw], slot["probs"][k, :nw], stream=ks,
                          workspace=slot["m_ws"])
            # model k's window w at probs[k * max_windows * L + w * L]
            _lib.check(_lib.lib().aa_track_mean(
                _lib.dptr(slot["probs"]), len(self.models), self.max_windows * self.L, self.L,
                _lib.dptr(slot["d_tr"][0]), _lib.dptr(slot["d_tr"][1]), nt, _lib.dptr(slot["means"]),
                _lib.stream_ptr(ks)), "aa_track_mean")
            with torch.cuda.stream(ks):
                slot["h_means"][:nt].copy_(slot["means"][:nt], non_blocking=True)
        slot["done"].record(ks)
        slot["pending"] = owners

    def _drain(self, slot):
        if slot["pending"] is None:
            return
        slot["done"].synchronize()
        owners, slot["pending"] = slot["pending"], None
        means = slot["h_means"].numpy()
        for i, (key, ti) in enumerate(owners):
            yield key, ti, means[i].copy()
