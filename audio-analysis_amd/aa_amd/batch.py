"""Batched corpus analysis: K recordings per GPU pass (BASELINE configs[3]).

The reference analyses one recording per process (``analyse.py FILE``,
src/analyse.py:434-470 -> classify(), src/identify_tracks.py:416-573).  Per
file that is decode, get_end, signal_noise, the track builder, the front end
and the models over the tracks' windows, and the post-processing to JSON.
On the GPU every one of those device steps is small for a single 60 s file
(tens of microseconds), so running them file by file leaves the device idle
behind launch latencies and blocking readbacks.  Here a rank takes its files
K at a time:

  * decode: worker threads read each PCM16 48 kHz WAV straight into a pinned
    host slot (other formats and rates go through ``load_recording``); the
    batch crosses PCIe as int16 and ``aa_pcm_s16_to_f32`` widens it on the
    device exactly as the host decode would;
  * get_end: one ``aa_span_nonzero`` launch over every file's chunk spans,
    one readback;
  * signal_noise: ``aa_sn_run_batch`` -- per file the STFT / medians / mask
    launches back to back, then one morphology + components pass for the
    whole batch -- into per-file result slots, one readback of the counts and
    component rows;
  * tracks: host, per file (as the reference);
  * classify: ``Classifier.classify_batch`` -- one front-end launch set over
    every file's windows, one forward per model, one track mean, one copy;
  * post-processing (``analyse.species_result``) on a host thread while the
    next batch runs on the device.

Each file's result is the document ``analyse.examine`` writes for it alone,
byte for byte (tests/test_gpu_batch.py): numpy's global RandomState is
reseeded per file right before its window schedule, exactly as the per-file
corpus path seeds it before ``examine``.
"""
from __future__ import annotations

import logging
import os
import struct
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib

SR = 48000


@dataclass
class Decoded:
    """A decoded recording: ``s16`` (interleaved int16 samples as a view of a
    pinned slot, ``channels`` of them per frame) or ``f32`` (mono samples at
    ``sr_in``, resampled to 48 kHz on the device as they are uploaded; parity
    unpinned for those: aa_amd.resample is held to libsoxr HQ's specification,
    not to its samples, see its header)."""
    n: int                   # frames at 48 kHz
    sr: int                  # 48000
    s16: object = None       # numpy int16 [n * channels] (view into a pinned slot)
    s16_t: object = None     # the same bytes as a pinned torch int16 tensor
    channels: int = 1
    f32: object = None       # numpy float32 [n_in] at sr_in
    sr_in: int = SR
    slot: int = -1
    dev: object = None       # the recording's samples in the batch's device PCM

    def frames(self):
        """Host float32 samples at 48 kHz (only band-pass filtered tracks need them)."""
        if self.f32 is None:
            from .audio import _to_mono
            self.f32 = _to_mono(np.asarray(self.s16), self.channels)
        if self.sr_in != SR:
            return self.dev.cpu().numpy()
        return self.f32


def _wav_pcm16(buf: np.ndarray, size: int):
    """(data offset, data bytes, channels, sr) if buf[:size] is a PCM16 RIFF/WAVE
    file, else None (decode() handles everything else)."""
    b = buf[:min(size, 1 << 16)].tobytes()
    if len(b) < 12 or b[:4] != b"RIFF" or b[8:12] != b"WAVE":
        return None
    pos, fmt = 12, None
    while pos + 8 <= size:
        if pos + 8 > len(b):
            b = buf[:min(size, pos + (1 << 16))].tobytes()
        cid, csz = b[pos:pos + 4], struct.unpack("<I", b[pos + 4:pos + 8])[0]
        if cid == b"fmt ":
            if pos + 8 + 16 > len(b):
                return None
            fmt = struct.unpack("<HHIIHH", b[pos + 8:pos + 24])
            if fmt[0] == 0xFFFE and csz >= 26 and pos + 34 <= len(b):
                fmt = (struct.unpack("<H", b[pos + 32:pos + 34])[0],) + fmt[1:]
        elif cid == b"data":
            if fmt is None:
                return None
            tag, ch, sr, _, _, bits = fmt
            if tag != 1 or bits != 16 or not 1 <= ch <= 8 or (pos + 8) % 2:
                return None
            n = min(csz, size - pos - 8)
            return pos + 8, n // (2 * ch) * 2 * ch, ch, sr
        pos += 8 + csz + (csz & 1)
    return None


class SlotPool:
    """Pinned host slots, each holding one file's bytes (one per recording in
    flight: the prefetch depth plus the batches on the device)."""

    def __init__(self, n_slots: int, slot_bytes: int):
        import threading
        self.bytes = int(slot_bytes)
        self.t, self.np, self.free = [], [], []
        self._cv = threading.Condition()
        self.grow(n_slots)

    def grow(self, n_slots: int):
        with self._cv:
            while len(self.t) < n_slots:
                self.t.append(torch.empty(self.bytes, dtype=torch.uint8, pin_memory=True))
                self.np.append(self.t[-1].numpy())
                self.free.append(len(self.t) - 1)
                self._cv.notify()

    def get(self) -> int:
        with self._cv:
            while not self.free:
                self._cv.wait()
            return self.free.pop()

    def put(self, i: int):
        with self._cv:
            self.free.append(i)
            self._cv.notify()


def decode_into(path, pool: SlotPool):
    """Decode one file; PCM16 48 kHz WAV lands in a pinned slot untouched.
    The file comes in with one aa_read_file call (stat, open, read, close
    without the interpreter lock: the decoder threads otherwise queued for it
    behind the lanes' Python at every step)."""
    import ctypes as C
    from . import identify_tracks as it
    i = pool.get()
    got = C.c_int64(0)
    rc = _lib.lib().aa_read_file(os.fsencode(path), pool.t[i].data_ptr(), pool.bytes, C.byref(got))
    if rc == _lib.AA_ERR_INVALID:
        pool.put(i)
        raise OSError(_lib.lib().aa_last_error().decode(errors="replace"))
    if rc == _lib.AA_OK:
        try:
            buf = pool.np[i]
            w = _wav_pcm16(buf, got.value)
            if w is not None and w[3] == SR:
                off, nb, ch, sr = w
                t = pool.t[i][off:off + nb].view(torch.int16)
                return Decoded(n=nb // (2 * ch), sr=sr, s16=buf[off:off + nb].view(np.int16), s16_t=t,
                               channels=ch, slot=i)
        except Exception:
            pool.put(i)
            raise
    pool.put(i)  # (larger than a slot, or not a 48 kHz PCM16 WAV)
    # FLAC, other WAV encodings; other rates are resampled on the device at upload
    frames, sr = it.load_recording(str(path), resample=None)
    from .resample import out_length
    return Decoded(n=out_length(len(frames), sr, SR), sr=SR, f32=np.ascontiguousarray(frames, dtype=np.float32),
                   sr_in=sr)


class _Laps:
    """Wall time per host phase of the batch loop (AA_BATCH_PROFILE=1 prints it;
    AA_BATCH_TRACE=path also keeps every (thread, phase, start, end) interval,
    CLOCK_MONOTONIC ns like rocprofv3's kernel trace, written there as JSON)."""

    def __init__(self):
        self.t = {}
        self.cpu = {}  # the calling thread's CPU time per phase (time.thread_time)
        self._c0 = {}
        self.events = [] if os.environ.get("AA_BATCH_TRACE") else None

    def lap(self, name, t0):
        import threading
        t1 = time.perf_counter()
        self.t[name] = self.t.get(name, 0.0) + (t1 - t0)
        tid = threading.get_ident()
        c1 = time.thread_time()
        if tid in self._c0:
            self.cpu[name] = self.cpu.get(name, 0.0) + (c1 - self._c0[tid])
        self._c0[tid] = c1
        if self.events is not None:
            import threading
            now = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
            self.events.append((threading.get_ident(), name, now - int((t1 - t0) * 1e9), now))
        return t1

    def report(self):
        return " ".join(f"{k}={1e3 * v:.1f}ms (cpu {1e3 * self.cpu.get(k, 0.0):.1f})" for k, v in self.t.items())


@dataclass
class _Rec:
    idx: int
    path: str
    dec: Decoded
    meta: object
    off: int = 0
    length: float = 0.0
    signals: list = field(default_factory=list)
    tracks: list = field(default_factory=list)
    res: object = None
    err: object = None


class _Lane:
    """One batch in flight: its own HIP stream and every device buffer a batch
    touches (PCM, int16 staging, signal_noise workspace and result slots, the
    front-end / model workspaces), so two host threads can each drive a batch:
    while one waits on its readbacks the other runs its host steps, and the
    device overlaps the two batches' kernels."""

    def __init__(self, dev):
        self.dev = dev
        self.stream = torch.cuda.Stream(device=dev)
        self.copy = torch.cuda.Stream(device=dev)
        self.pcm = torch.empty(0, dtype=torch.float32, device=dev)
        self.s16 = torch.empty(0, dtype=torch.int16, device=dev)
        self.sn_ws = None
        self.sn_buf = None
        self.ws = {}  # classify_batch workspaces

    def buffers(self, n_f32, n_s16):
        if self.pcm.numel() < n_f32:
            self.pcm = torch.empty(int(n_f32 * 1.25) + 1, dtype=torch.float32, device=self.dev)
        if self.s16.numel() < n_s16:
            self.s16 = torch.empty(int(n_s16 * 1.25) + 1, dtype=torch.int16, device=self.dev)
        return self.pcm, self.s16


SN_CAP = 4096   # components per recording kept in the batch slots
PREFETCH = 2    # batches decoded ahead of the newest batch a lane has taken
_SN_LOCK = __import__("threading").Lock()
SN_HEAD = 64    # component rows read back with the counts (more: a second copy)

_POOLS = {}


def slot_pool(n_slots, slot_bytes):
    """Pinned slots persist across runs (allocating pinned memory is slow):
    one grow-only pool per slot size class."""
    size = -(-int(slot_bytes) // (1 << 20)) << 20
    pool = _POOLS.get(size)
    if pool is None:
        pool = _POOLS[size] = SlotPool(0, size)
    pool.grow(n_slots)
    return pool


class BatchAnalyser:
    """examine() for many files of one rank, K per device pass, ``lanes``
    batches in flight."""

    def __init__(self, bird_models, analyse_tracks=False, device=None, precision=None, batch=16, workers=8,
                 lanes=2):
        from .identify_tracks import _group_models
        from .pipeline import Classifier
        self.bird_models = bird_models
        self.analyse_tracks = bool(analyse_tracks)
        self.dev = torch.device(device or "cuda")
        self.K = int(batch)
        self.workers = int(workers)
        self.n_lanes = max(1, int(lanes))
        self.groups = _group_models(bird_models) if bird_models is not None else None
        self.clf = Classifier.shared(precision=precision, device=self.dev)
        self.timing = _Laps()

    # ---- one batch --------------------------------------------------------
    def _upload(self, lane, recs):
        """PCM of the batch into one device f32 buffer (recording r at r.off)."""
        total = sum(r.dec.n for r in recs)
        n16 = sum(r.dec.n * r.dec.channels for r in recs if r.dec.s16 is not None)
        pcm, s16 = lane.buffers(total, n16)
        cur = torch.cuda.current_stream(self.dev)
        lane.copy.wait_stream(cur)  # the lane's previous batch is done with both buffers
        off = o16 = 0
        with torch.cuda.stream(lane.copy):
            for r in recs:
                r.off = off
                d = r.dec
                if d.s16 is not None:
                    s16[o16:o16 + d.s16_t.numel()].copy_(d.s16_t, non_blocking=True)
                    d.o16 = o16
                    o16 += d.s16_t.numel()
                elif d.sr_in == SR:
                    pcm[off:off + d.n].copy_(torch.from_numpy(d.f32), non_blocking=False)
                off += d.n
        cur.wait_stream(lane.copy)
        L = _lib.lib()
        from .resample import resample_device
        # every recording mono PCM16: the int16 and f32 offsets coincide, so one
        # widening launch covers the batch
        mono16 = all(r.dec.s16 is not None and r.dec.channels == 1 for r in recs)
        if mono16 and total:
            _lib.check(L.aa_pcm_s16_to_f32(_lib.dptr(s16), total, 1, _lib.dptr(pcm), _lib.stream_ptr(cur)),
                       "aa_pcm_s16_to_f32")
        for r in recs:
            d = r.dec
            d.dev = pcm[r.off:r.off + d.n]
            if mono16:
                continue
            if d.s16 is not None and d.n:
                _lib.check(L.aa_pcm_s16_to_f32(_lib.dptr(s16) + 2 * d.o16, d.n, d.channels,
                                               _lib.dptr(pcm) + 4 * r.off, _lib.stream_ptr(cur)),
                           "aa_pcm_s16_to_f32")
            elif d.s16 is None and d.sr_in != SR:  # librosa.resample to 48 kHz (aa_amd.resample)
                resample_device(torch.from_numpy(d.f32).to(self.dev), d.sr_in, SR, out=d.dev)
        return pcm[:total]

    def _get_end(self, pcm, recs):
        """get_end (src/identify_tracks.py:387-413) of every recording, one launch."""
        from .gpu_ops import get_end_spans
        spans, owner, starts = [], [], []
        for k, r in enumerate(recs):
            sp, st, hop = get_end_spans(r.dec.n, r.dec.sr)
            r.length = r.dec.n / r.dec.sr
            if len(st):
                spans.append(sp + r.off)
                owner += [k] * len(st)
                starts += st
        if not spans:
            return
        sp = torch.from_numpy(np.concatenate(spans)).to(self.dev)
        flags = torch.empty(len(owner), dtype=torch.int32, device=self.dev)
        _lib.check(_lib.lib().aa_span_nonzero(_lib.dptr(pcm), int(pcm.numel()), _lib.dptr(sp), len(owner),
                                              _lib.dptr(flags), _lib.stream_ptr()), "aa_span_nonzero")
        f = flags.cpu().numpy()
        seen = set()
        for j in np.flatnonzero(f == 0):
            k = owner[j]
            if k not in seen:  # the first constant chunk of recording k
                seen.add(k)
                recs[k].length = starts[j] * 281 // recs[k].dec.sr

    def _signal_noise(self, lane, pcm, recs):
        """signal_noise (src/identify_tracks.py:650-706) of every recording:
        aa_sn_run_batch over up to 64 recordings at a time (per recording the
        STFT / medians / mask launches, then one morphology + components pass
        for all of them) into per-recording slots [1 + SN_CAP][6] int32 (row 0:
        count, status), one readback of every slot's head."""
        import ctypes as C
        from .identify_tracks import Signal
        from .signals import detector
        by_sr = {}
        for k, r in enumerate(recs):
            by_sr.setdefault(r.dec.sr, []).append(k)
        L = _lib.lib()
        for sr, ks in by_sr.items():
            det = detector(sr, 281, self.dev)
            nsig = [int(sr * recs[k].length) for k in ks]
            K = min(len(ks), 64)
            need = L.aa_sn_batch_workspace_bytes(det._h, max(nsig), K)
            if lane.sn_ws is None or lane.sn_ws.numel() < need:
                lane.sn_ws = torch.empty(need, dtype=torch.uint8, device=self.dev)
            if lane.sn_buf is None or lane.sn_buf.shape[0] < len(ks):
                lane.sn_buf = torch.empty((len(ks), 1 + SN_CAP, 6), dtype=torch.int32, device=self.dev)
            buf, ws = lane.sn_buf, lane.sn_ws
            for c0 in range(0, len(ks), 64):
                part = ks[c0:c0 + 64]
                offs = (C.c_int64 * len(part))(*[recs[k].off if nsig[c0 + j] else 0 for j, k in enumerate(part)])
                lens = (C.c_int64 * len(part))(*nsig[c0:c0 + len(part)])
                _lib.check(L.aa_sn_run_batch(det._h, _lib.dptr(pcm), offs, lens, len(part), _lib.dptr(ws), ws.numel(),
                                             _lib.dptr(buf[c0, 1:]), SN_CAP, 1 + SN_CAP, _lib.dptr(buf[c0, 0]),
                                             (1 + SN_CAP) * 6, _lib.stream_ptr()), "aa_sn_run_batch")
            head = buf[:len(ks), :1 + SN_HEAD].cpu().numpy()
            for j, k in enumerate(ks):
                c, status = int(head[j, 0, 0]), int(head[j, 0, 1])
                if status & _lib.AA_SN_NONFINITE:
                    recs[k].err = ValueError("Audio buffer is not finite everywhere")  # librosa valid_audio
                    continue
                if status & _lib.AA_SN_RUN_OVERFLOW or c > SN_CAP:
                    # more components than a slot holds: this recording alone,
                    # through the detector's own (shared) buffers
                    try:
                        with _SN_LOCK:
                            stats = det.components(pcm[recs[k].off:recs[k].off + nsig[j]])
                    except Exception as e:
                        recs[k].err = e
                        continue
                else:
                    rows = head[j, 1:1 + c] if c <= SN_HEAD else buf[j, 1:1 + c].cpu().numpy()
                    rows = rows.astype(np.int64)
                    stats = rows[np.lexsort((rows[:, 5], rows[:, 0]))][:, :5]
                recs[k].signals = [Signal(*tu) for tu in det.to_tuples(stats)]

    def _classify(self, lane, pcm, recs):
        from .identify_tracks import MAX_FRQUENCY, Signal, tracks_from_signals
        from .pipeline import BatchRec
        todo = []
        for r in recs:
            if r.err is not None:
                continue
            raw_length = r.dec.n / r.dec.sr
            if self.analyse_tracks:
                if r.meta is None:
                    r.res = None
                    continue
                tracks = []
                for t in r.meta["Tracks"]:
                    s = Signal(t["start"], t["end"], t.get("minFreq", 0), t.get("maxFreq", MAX_FRQUENCY))
                    s.track_id = t["id"]
                    tracks.append(s)
            else:
                tracks = tracks_from_signals(r.signals, r.length)
            if len(tracks) == 0:
                r.res = ([], r.length, [], raw_length, [])
                continue
            r.tracks = tracks
            todo.append(r)
        if not todo:
            return
        brs = [BatchRec(n=r.dec.n, off=r.off, tracks=r.tracks, frames=r.dec.frames, seed=r.idx) for r in todo]
        out = self.clf.classify_batch(pcm, SR, brs, self.groups, ws=lane.ws)
        for r, o in zip(todo, out):
            if isinstance(o, BaseException):
                r.err = o
            else:
                r.res = (r.tracks, r.length, r.signals, r.dec.n / r.dec.sr, list(o))

    def _finish(self, recs, t0):
        from .analyse import species_result
        from .corpus import FAILED
        out = {}
        dt = round((time.time() - t0) / max(len(recs), 1), 1)
        for r in recs:
            if r.err is not None:
                logging.error("%s: %s", r.path, r.err)
                out[r.idx] = {FAILED: f"{type(r.err).__name__}: {r.err}"}
                continue
            doc = species_result(r.res, r.meta, self.analyse_tracks, self.bird_models is not None)
            doc["processing_time_seconds"] = dt
            out[r.idx] = doc
        return out

    def process(self, items, lane, pool=None):
        """items: [(file_idx, path, Decoded | Exception, sidecar meta)] -> {file_idx: document}."""
        t0 = time.time()
        recs, failed = [], []
        for idx, path, dec, meta in items:
            if isinstance(dec, BaseException):
                failed.append(_Rec(idx, str(path), None, meta, err=dec))
            else:
                recs.append(_Rec(idx, str(path), dec, meta))
        if recs:
            try:
                with torch.cuda.stream(lane.stream):
                    tm = self.timing
                    t = time.perf_counter()
                    pcm = self._upload(lane, recs)
                    t = tm.lap("upload", t)
                    self._get_end(pcm, recs)
                    t = tm.lap("get_end", t)
                    self._signal_noise(lane, pcm, recs)
                    t = tm.lap("signal_noise", t)
                    self._classify(lane, pcm, recs)
                    tm.lap("classify", t)
            finally:
                # (the slots stay held until here: band-pass filtered tracks
                # read a recording's host samples during classify)
                if pool is not None:
                    for r in recs:
                        if r.dec.slot >= 0:
                            pool.put(r.dec.slot)
                            r.dec.slot = -1
        t = time.perf_counter()
        docs = self._finish(recs + failed, t0)
        self.timing.lap("post", t)
        return docs

    def run(self, jobs):
        """jobs: [(file_idx, path)] -> {file_idx: document} (the files of this rank)."""
        import threading
        from .analyse import read_sidecar
        if not jobs:
            return {}
        if self.bird_models is None:  # examine() without models reads no audio
            from .analyse import species_result
            return {i: dict(species_result(None, read_sidecar(p), self.analyse_tracks, False),
                            processing_time_seconds=0.0) for i, p in sorted(jobs)}
        K = self.K
        lanes = [_Lane(self.dev) for _ in range(min(self.n_lanes, -(-len(jobs) // K)))]
        slot_bytes = max(os.path.getsize(p) for _, p in jobs) + 4096
        # slots: every lane's batch plus PREFETCH batches decoded ahead of the
        # newest batch a lane has taken -- exactly the batches that can hold
        # slots at once, so a decode never waits for a slot (a waiting decode
        # of a later batch could otherwise hold the slots the oldest batch needs)
        pool = slot_pool(min(len(jobs), (len(lanes) + PREFETCH) * K), slot_bytes)

        def load(job):
            idx, path = job
            meta = None
            try:
                meta = read_sidecar(path)
                return idx, path, decode_into(path, pool), meta
            except Exception as e:
                logging.error("Could not load %s", path, exc_info=True)
                return idx, path, Exception(f"Could not load {path}") if not isinstance(e, ValueError) else e, meta

        results, errors = {}, []
        lock = threading.Lock()
        batches = [jobs[b:b + K] for b in range(0, len(jobs), K)]
        with ThreadPoolExecutor(max_workers=self.workers) as io:
            futs = {}  # batch index -> its decode futures, submitted PREFETCH batches ahead
            state = {"next": 0, "submitted": 0}

            def submit_upto(b):
                while state["submitted"] < min(b, len(batches)):
                    futs[state["submitted"]] = [io.submit(load, j) for j in batches[state["submitted"]]]
                    state["submitted"] += 1

            def worker(lane):
                torch.cuda.set_device(self.dev)
                prof = None
                if os.environ.get("AA_BATCH_CPROFILE"):  # host-side profile of this lane (tools)
                    import cProfile
                    # AA_BATCH_CPROFILE_CPU=1: the lane thread's CPU time (what
                    # holds the GIL) instead of wall time (GPU waits included)
                    cpu = os.environ.get("AA_BATCH_CPROFILE_CPU") == "1"
                    prof = cProfile.Profile(time.thread_time) if cpu else cProfile.Profile()
                    prof.enable()
                try:
                    while True:
                        with lock:
                            b = state["next"]
                            if b >= len(batches):
                                return
                            state["next"] += 1
                            submit_upto(b + 1 + PREFETCH)
                            fb = futs.pop(b)
                        t = time.perf_counter()
                        items = [f.result() for f in fb]
                        self.timing.lap("wait_decode", t)
                        docs = self.process(items, lane, pool)
                        with lock:
                            results.update(docs)
                except BaseException as e:  # surfaces in the caller
                    errors.append(e)
                finally:
                    if prof is not None:
                        prof.disable()
                        prof.dump_stats(f"{os.environ['AA_BATCH_CPROFILE']}.{time.monotonic_ns()}")

            with lock:
                submit_upto(len(lanes) + PREFETCH)
            threads = [threading.Thread(target=worker, args=(ln,), daemon=True) for ln in lanes]
            for th in threads:
                th.start()
            for th in threads:
                th.join()
        for ln in lanes:
            ln.stream.synchronize()
        if errors:
            raise errors[0]
        if os.environ.get("AA_BATCH_PROFILE"):
            logging.warning("batch phases over %d files (%d lanes): %s", len(jobs), len(lanes), self.timing.report())
        if self.timing.events is not None:
            import json
            with open(os.environ["AA_BATCH_TRACE"], "w") as f:
                json.dump(self.timing.events, f)
        return dict(sorted(results.items()))
