"""Throughput benchmark of the MI355X hot path (BASELINE.json metric).

Workload (BASELINE.json configs[1], "config 2"): one step = one batch of 64
analysis windows -- 39 windows of a 60 s clip + 25 windows of a second 60 s
clip (48 kHz mono, synthetic, int16-quantised; reference stride 1.5 s / length
3 s) -- through the GPU log-mel front end (htk custom mel, n_fft 4096, hop 640,
160 bands, power_to_db) and the model1 CNN, then the per-track mean.  PCM and
window tables are resident in HBM before the timed region; the steps rotate
over 4 resident clip pairs (kernel times depend on the data).  Two batches
are in flight on two HIP streams, steps alternating between them (--pipeline
0: one stream, back to back, the 'serial' secondary).

Headline precision: split-bf16 ("bf16x3", classify()'s default), the fastest
mode that holds the north-star gate max|delta logit| <= 1e-3 against the CPU
oracle -- asserted here on the step's 64 windows.  At N=1 the same line carries
secondary measurements: f32 MFMA (also gated), bf16 and fp8 (throughput modes,
delta reported), and the headline mode on cold PCM (a fresh clip pair per
step from a pool larger than the 256 MiB Infinity Cache, alternated with the
headline step three times).

Audio-seconds per step: a 60 s clip is covered by 39 windows, so each window
counts 60/39 s; value = (windows processed by all ranks x 60/39) / max-over-
ranks wall time.  Multi-GPU: one process per GPU (torchrun, or ``--gpus N``
which spawns the N ranks itself), each with its own clips (weak scaling); the
only collective is the final RCCL all-gather of per-track results (§8e).
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import socket
import sys
import tempfile
import time
from pathlib import Path

# hardware queues per process: HIP maps streams onto them round-robin, and two
# streams on one queue run back to back.  The corpus path keeps 8 lanes x
# (compute + copy) streams busy; HIP's default of 4 queues makes them share
# (configs[3] secondary 114-121k with 4 queues / 3 lanes, 130-149k with 16 /
# 8, same box; profiles/r06/corpus_queues_lanes.txt).  Raised, never lowered
# (a value above 16 that the environment set stays), and read once, at HIP's
# initialisation: before anything below touches the GPU.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

ROOT = Path(__file__).resolve().parent
for p in (str(ROOT), str(ROOT / "audio-analysis_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np
import torch
import torch.distributed as dist

METRIC = "audio-seconds classified/sec/GPU on 60 s mono; max|delta logit| vs CPU ref"
WINDOWS_PER_CLIP = 39
SECONDS_PER_WINDOW = 60.0 / WINDOWS_PER_CLIP
BATCH_A, BATCH_B = 39, 25
LOGIT_GATE = 1e-3
GATED = ("bf16x3", "f32")
# dense MFMA TFLOP/s, MI355X_MICROARCH.md.  bf16x3 issues three bf16 MFMAs per
# f32-accurate MAC, so its ceiling for the algorithmic FLOPs is a third of the
# bf16 peak.  fp8: the dtype's dense peak, reached only by the block-scaled
# K=128 form; the non-scaled 16x16x32 fp8 MFMA the kernels use issues at the
# bf16 rate.
PEAK = {"bf16": 2500.0, "bf16x3": 2500.0 / 3, "f32": 157.3, "fp8": 5000.0}
VALU_F32_PEAK = 157.3                   # FP32 VALU TFLOP/s (fma counted as 2)
VALU_F64_PEAK = 78.6                    # FP64 VALU TFLOP/s (AMD MI355X spec; half the FP32 vector rate)
HBM_PEAK_GBS = 8000.0
WORKLOAD = ("config2: 64 windows/step (39 of clip A + 25 of clip B, 60 s 48 kHz mono), "
            "htk log-mel n_fft 4096 hop 640 160 mel + model1 CNN")
# --model effnetv2: the "efficientnet" route of classify() (reference
# src/identify_tracks.py:539-540: the log-mel repeated to 3 channels) through
# an EfficientNetV2-B0-shaped graph (tools/make_models.graph_arch) on the graph
# executor, hop 281 (T = 513)
WORKLOADS = {"model1": WORKLOAD,
             "effnetv2": ("config2-effnetv2: 64 windows/step (39 of clip A + 25 of clip B, 60 s 48 kHz mono), "
                          "htk log-mel n_fft 4096 hop 281 160 mel x3 channels + EfficientNetV2-B0-shaped graph")}
CORPUS_POOL = 64  # distinct WAV files per rank of the configs[3] run (cycled)
COLD_POOL = 16  # clip pairs of the cold-PCM variant: 16 x 23 MB > the 256 MiB Infinity Cache
# clip pairs the headline rotates over (resident, 92 MB: inside the Infinity
# Cache): kernel times depend on the data (MFMA power and clock), and one
# pair alone measured 7 % faster than the average of four
HEAD_PAIRS = 4


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks; without torchrun's env, bench.py spawns one process per GPU itself")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="model1", choices=sorted(WORKLOADS),
                    help="model1: the build-defined sparrow-style CNN (headline); effnetv2: an EfficientNetV2-B0-"
                         "shaped graph on 3-channel log-mel (the efficientnet route)")
    ap.add_argument("--precision", default="bf16x3", choices=["bf16x3", "f32", "bf16", "fp8"],
                    help="bf16x3: split-bf16 (gated, default); fp8: OCP e4m3fn CNN (BASELINE configs[4])")
    ap.add_argument("--logmel", default="f32", choices=["f32", "f16"],
                    help="log-mel dtype between the front end and the CNN (f16: BASELINE configs[4])")
    ap.add_argument("--secondary", default="serial,f32,bf16,fp8,fp8_f16mel,cold,config3,config4,effnetv2",
                    help="N=1 only: extra modes measured into the same line ('' disables)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="bound on the CPU-baseline sample (0 disables)")
    ap.add_argument("--cpu-workers", type=int, default=16,
                    help="CPU-baseline processes for the numpy front end (the GPU box's CPU share is 16)")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--pipeline", type=int, default=2, choices=[0, 1, 2, 3, 4],
                    help="2 (default): two batches in flight on two HIP streams, steps alternating between "
                         "them (each step: front end -> CNN -> track mean of its own batch; 3, 4: as many "
                         "streams); 1: only the "
                         "front end of batch k+1 on a second stream beside the CNN of batch k; 0: one stream, "
                         "back to back (reported as the 'serial' secondary)")
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4],
                    help="2: the 64-window step (BASELINE configs[1], the headline); 3: streamed 60 s clips "
                         "through the model1+2+3 ensemble (configs[2]), PCM uploaded from pinned host memory; "
                         "4: a corpus of 60 s WAV files through the whole analyse path (configs[3])")
    ap.add_argument("--clips", type=int, default=1000, help="--config 3: clips per rank")
    ap.add_argument("--files", type=int, default=1250,
                    help="--config 4: files per rank (BASELINE configs[3]: 10k clips over 8 GPUs)")
    ap.add_argument("--batch", type=int, default=32,
                    help="--config 4: recordings per device pass (aa_amd.batch); 0 = one file at a time")
    ap.add_argument("--procs-per-gpu", type=int, default=1,
                    help="--config 4: host processes feeding each GPU (the host steps the reference runs in "
                         "Python -- decode, tracks, JSON -- scale with processes, not threads); ranks sharing "
                         "a GPU gather over gloo.  --config 2: ranks sharing one GPU over gloo (rehearses the "
                         "N-rank path -- per-rank parity gate, max-over-ranks time, record gather -- on one GPU)")
    return ap.parse_args(argv)


def fe_settings(model="model1"):
    from aa_amd.frontend import FeSettings
    if model == "effnetv2":
        return FeSettings(htk=True, hop_length=281, n_fft=4096, n_mels=160, break_freq=1750, channels=3)
    return FeSettings(htk=True, hop_length=640, n_fft=4096, n_mels=160, break_freq=1750)


def fe_config(s):
    """oracle.fe_oracle config of a FeSettings."""
    return dict(sr=s.sr, hop_length=s.hop_length, n_mels=s.n_mels, fmin=s.fmin, fmax=s.fmax, n_fft=s.n_fft,
                power=s.power, db_scale=s.db_scale, htk=s.htk, break_freq=s.break_freq,
                normalize=s.normalize, mean_sub=s.mean_sub, channels=s.channels, win_len=s.win_len)


def window_samples(pcm, view, win_len):
    """The window a view (src, n_valid, pad_left) denotes, as a 1-D array."""
    s, n, p = view
    w = np.zeros(win_len, np.float32)
    w[p:p + n] = pcm[s:s + n]
    return w


def make_batch(rank, fe_settings, pair=0):
    """Two resident 60 s clips and the 64-window table (39 + 25)."""
    from aa_amd.frontend import pack_windows
    from aa_amd.windows import track_windows
    from tools import synth
    base = 2 * (rank * 1000 + pair)
    a, b = synth.clip(base), synth.clip(base + 1)
    pcm = np.concatenate([a, b])
    sr = fe_settings.sr
    va = track_windows(len(a), sr, 0.0, 60.0, 60.0, 0, 24000, 3, 1.5, 50, 11000)
    vb = track_windows(len(b), sr, 0.0, 60.0, 60.0, 0, 24000, 3, 1.5, 50, 11000)[:BATCH_B]
    assert len(va) == BATCH_A
    rows = np.concatenate([pack_windows(va, len(a)), pack_windows(vb, len(b), offset=len(a))])
    views = [(s, n, p) for (s, n, p) in va] + [(s + len(a), n, p) for (s, n, p) in vb]
    return pcm, rows, views


def _fe_worker(job):
    from oracle import fe_oracle
    windows, cfg = job
    return [fe_oracle.window_logmel(w, cfg) for w in windows]


def cpu_baseline(pcm, views, model_path, cfg, budget_s, workers):
    """Oracle on the host cores: numpy librosa-0.11 restatement of the front end
    over a process pool of ``workers`` (spawned: the parent holds a GPU
    context) + torch-CPU fp32 model1 on ``workers`` threads, on a bounded
    sample -- passes over the step's windows, 32 at a time, until ``budget_s``
    seconds of CPU work are done.  Returns (audio-s/s, windows, seconds)."""
    import multiprocessing as mp
    from oracle import cnn_oracle
    torch.set_num_threads(workers)
    ctx = mp.get_context("spawn")
    with ctx.Pool(workers) as pool:
        warm = [window_samples(pcm, views[0], cfg["win_len"])]
        pool.map(_fe_worker, [(warm, cfg)] * workers)  # import warm-up
        t0 = time.perf_counter()
        done = 0
        while done == 0 or (time.perf_counter() - t0) < budget_s:
            i = done % len(views)
            chunk = views[i:i + 32]
            wins = [window_samples(pcm, v, cfg["win_len"]) for v in chunk]
            jobs = [(wins[k::workers], cfg) for k in range(min(workers, len(wins)))]
            parts = pool.map(_fe_worker, jobs)
            mels = [None] * len(wins)
            for k, part in enumerate(parts):
                mels[k::workers] = part
            cnn_oracle.forward(model_path, np.stack(mels))
            done += len(chunk)
        dt = time.perf_counter() - t0
    return done * SECONDS_PER_WINDOW / dt, done, dt


def reference_logits(pcm, views, model_path, cfg):
    """Oracle logits of the step's windows (the parity check of the line)."""
    from oracle import cnn_oracle, fe_oracle
    mels = np.stack([fe_oracle.window_logmel(window_samples(pcm, v, cfg["win_len"]), cfg) for v in views])
    return cnn_oracle.forward(model_path, mels)[0]


def load_traffic(n_dispatch, precision, workload=WORKLOAD):
    """HBM bytes per launch of each kernel of one step, in dispatch order, from
    the committed rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE summary of this same
    workload (tools/pmc_traffic.py; FETCH_SIZE doubled per
    MI355X_MICROARCH.md).  None when no summary of this workload exists."""
    for path in sorted((ROOT / "profiles").glob("*/pmc_traffic*.json"), reverse=True):
        try:
            d = json.loads(path.read_text())
        except (OSError, ValueError):
            continue
        if (d.get("workload") == workload and d.get("precision", "bf16") == precision
                and len(d.get("kernels", [])) == n_dispatch):
            return d, path.relative_to(ROOT).as_posix()
    return None, None


def load_profiled_stages(traffic, precision):
    """Average duration (us) of each launch of one step from the committed
    rocprofv3 --kernel-trace --stats summary of the serial step
    (bench_kernel_stats_serial_<precision>.csv beside the PMC summary),
    launches named by the PMC summary's per-dispatch kernel list; a launch that
    dispatches a second kernel (the network tail's head_final) is charged both.
    None when either summary is missing."""
    if traffic is None:
        return None
    for path in sorted((ROOT / "profiles").glob(f"*/bench_kernel_stats_serial_{precision}.csv"), reverse=True):
        try:
            rows = list(csv.DictReader(path.open()))
        except OSError:
            continue
        avg = {r["Name"]: float(r["AverageNs"]) / 1e3 for r in rows}

        def find(name):
            hit = [v for k, v in avg.items() if k.startswith(name[:100])]
            return hit[0] if len(hit) == 1 else None

        durs = [find(k["name"]) for k in traffic["kernels"][:-1]]  # the last is track_mean
        if any(d is None for d in durs):
            continue
        head = find("aa::head_final")
        if head is not None:
            for i, k in enumerate(traffic["kernels"][:-1]):
                if "conv_tail" in k["name"]:
                    durs[i] += head
        return path.relative_to(ROOT).as_posix(), durs
    return None


# The lanes' HIP streams, shared by every Step of the process: HIP maps
# streams onto a few hardware queues (GPU_MAX_HW_QUEUES = 4) round-robin in
# creation order, and two lanes whose streams land on one queue run back to
# back -- a secondary measured after the headline had its two lanes on one
# queue (the efficientnet route 52k standalone, 41k as a secondary: its serial
# rate).  Reusing the headline's streams keeps every run's lanes on distinct
# queues.
_LANE_STREAMS = {}


def lane_stream(dev, j):
    key = (str(dev), j)
    if key not in _LANE_STREAMS:
        _LANE_STREAMS[key] = torch.cuda.Stream(device=dev)
    return _LANE_STREAMS[key]


class Step:
    """One configs[1] step on one device: FE -> model -> track mean, with the
    buffers of ``pairs`` resident clip pairs (1 = the headline; COLD_POOL =
    the cold-PCM variant, one pair per step in rotation)."""

    def __init__(self, dev, rank, model_path, precision, pairs=1, first=None, lm16=False, pipeline=False,
                 fe_s=None):
        from aa_amd.frontend import FrontEnd
        from aa_amd.model import Model
        self.fe_s = fe_s or fe_settings()
        lm_dtype = torch.float16 if lm16 else torch.float32  # configs[4]: fp16 log-mel
        self.fe = FrontEnd(self.fe_s, dev, out_dtype=lm_dtype)
        self.model = Model(model_path, (self.fe_s.n_mels, self.fe.T, self.fe_s.channels), precision=precision,
                           device=dev)
        batches = [first] if first is not None else []
        for k in range(len(batches), pairs):
            batches.append(make_batch(rank, self.fe_s, pair=k))
        self.pcm = [torch.from_numpy(b[0]).to(dev) for b in batches]
        self.rows = [torch.from_numpy(b[1]).to(dev) for b in batches]
        self.n_win = batches[0][1].shape[0]
        self.logmel = torch.empty(self.fe.out_shape(self.n_win), dtype=lm_dtype, device=dev)
        self.logits = torch.empty((self.n_win, self.model.n_labels), dtype=torch.float32, device=dev)
        self.probs = torch.empty_like(self.logits)
        self.wb = torch.tensor([0, BATCH_A], dtype=torch.int32, device=dev)
        self.wc = torch.tensor([BATCH_A, BATCH_B], dtype=torch.int32, device=dev)
        self.tmean = torch.empty((2, self.model.n_labels), dtype=torch.float32, device=dev)
        self.fe_ws = torch.empty(max(self.fe.workspace_bytes(self.n_win), 256), dtype=torch.uint8, device=dev)
        self.m_ws = torch.empty(max(self.model.workspace_bytes(self.n_win), 256), dtype=torch.uint8, device=dev)
        self.k = 0
        self.lanes = None
        if pipeline >= 2:
            # two batches in flight, each on its own stream (front end -> CNN ->
            # track mean), alternating steps: the kernels of one fill the other's
            # tails and phases
            self.lanes = []
            for j in range(int(pipeline)):
                self.lanes.append(dict(
                    s=lane_stream(dev, j), logmel=self.logmel if j == 0 else torch.empty_like(self.logmel),
                    fe_ws=self.fe_ws if j == 0 else torch.empty_like(self.fe_ws),
                    m_ws=self.m_ws if j == 0 else torch.empty_like(self.m_ws),
                    logits=self.logits if j == 0 else torch.empty_like(self.logits),
                    probs=self.probs if j == 0 else torch.empty_like(self.probs),
                    tmean=self.tmean if j == 0 else torch.empty_like(self.tmean)))
            self.pipeline = False
            return
        self.pipeline = bool(pipeline)
        if self.pipeline:
            # batch k+1's front end on s_fe into buffer (k+1) % 2 while the CNN
            # of batch k reads buffer k % 2 on the current stream
            self.s_fe = lane_stream(dev, "fe")
            self.lm2 = [self.logmel, torch.empty_like(self.logmel)]
            self.ws2 = [self.fe_ws, torch.empty_like(self.fe_ws)]
            self.fe_done = [torch.cuda.Event(), torch.cuda.Event()]
            self.cnn_done = [torch.cuda.Event(), torch.cuda.Event()]
            self.issued = -1  # last batch whose front end is issued

    def _fe_ahead(self, j):
        b = j % 2
        cur = torch.cuda.current_stream()
        self.s_fe.wait_event(self.cnn_done[b]) if j >= 2 else self.s_fe.wait_stream(cur)
        with torch.cuda.stream(self.s_fe):
            i = j % len(self.pcm)
            self.fe.run(self.pcm[i], self.rows[i], out=self.lm2[b], workspace=self.ws2[b])
            self.fe_done[b].record(self.s_fe)
        self.issued = j

    def __call__(self):
        from aa_amd.model import track_mean
        if self.lanes is not None:
            k = self.k
            self.k += 1
            L = self.lanes[k % len(self.lanes)]
            i = k % len(self.pcm)
            with torch.cuda.stream(L["s"]):
                self.fe.run(self.pcm[i], self.rows[i], out=L["logmel"], workspace=L["fe_ws"])
                self.model.forward(L["logmel"], L["logits"], L["probs"], workspace=L["m_ws"])
                track_mean(L["probs"][None], self.wb, self.wc, out=L["tmean"])
            self.logits, self.tmean = L["logits"], L["tmean"]
            return
        if self.pipeline:
            k = self.k
            self.k += 1
            if self.issued < k:
                self._fe_ahead(k)
            self._fe_ahead(k + 1)  # overlaps the CNN below
            b = k % 2
            cur = torch.cuda.current_stream()
            cur.wait_event(self.fe_done[b])
            self.model.forward(self.lm2[b], self.logits, self.probs, workspace=self.m_ws)
            self.cnn_done[b].record(cur)
            track_mean(self.probs[None], self.wb, self.wc, out=self.tmean)
            return
        i = self.k % len(self.pcm)
        self.k += 1
        self.fe.run(self.pcm[i], self.rows[i], out=self.logmel, workspace=self.fe_ws)
        self.model.forward(self.logmel, self.logits, self.probs, workspace=self.m_ws)
        track_mean(self.probs[None], self.wb, self.wc, out=self.tmean)

    def launches(self):
        return [(self.fe, i) for i in range(self.fe.n_stages())] + \
               [(self.model, i) for i in range(self.model.n_stages())]


def timed(step, steps, warmup, world):
    for _ in range(warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    return time.perf_counter() - t0


def collect(owner_stages, n_win):
    out = []
    for owner, i in owner_stages:
        name, flops, byts = owner.stage_info(i)
        ms, cnt = owner.stage_time(i)
        out.append(dict(owner=owner, idx=i, name=name, flops=flops * n_win, bytes=byts * n_win,
                        avg_ms=ms / max(cnt, 1), count=cnt))
    return out


def graph_stage_bound(name, flops, precision, nbytes=0.0):
    """(bound, peak, unit) of a model stage: MFMA convs against the
    precision's matrix peak -- or against HBM when their f32 activations take
    longer to stream at 8 TB/s than their MACs at the matrix peak (a 1x1 conv
    over 112 channels is memory-bound) -- exact-f32 VALU convs (conv_gf32_*)
    against the FP32 VALU peak, the memory-streaming graph nodes (depthwise
    convs, pools, add / multiply, affine, dense, matrix-vector) against HBM."""
    if name.startswith("conv_gf32"):
        if nbytes / (HBM_PEAK_GBS * 1e9) > flops / (VALU_F32_PEAK * 1e12):
            return "hbm", HBM_PEAK_GBS, "GB/s"
        return "valu", VALU_F32_PEAK, "TFLOP/s"
    if flops == 0 or name.startswith(("dwconv", "maxpool", "avgpool", "gmaxpool", "gavgpool", "add", "mul",
                                      "affine", "pow", "dense", "head", "pool", "matvec")):
        return "hbm", HBM_PEAK_GBS, "GB/s"
    if nbytes / (HBM_PEAK_GBS * 1e9) > flops / (PEAK[precision] * 1e12):
        return "hbm", HBM_PEAK_GBS, "GB/s"
    return "mfma", PEAK[precision], "TFLOP/s"


def stage_bound(name, precision):
    """(bound, peak, unit) of a launch stage by kernel name."""
    if name.startswith("fe_stft"):
        return "valu", VALU_F32_PEAK, "TFLOP/s"
    if name.startswith("sn_stft64"):
        return "valu_f64", VALU_F64_PEAK, "TFLOP/s"
    if name.startswith(("fe_", "sn_", "head", "pool", "track")):
        return "hbm", HBM_PEAK_GBS, "GB/s"
    return "mfma", PEAK[precision], "TFLOP/s"


def stage_table(owners, precision):
    """Per-stage time and roofline from HIP-event stage timing: owners =
    [(StageTiming object, items processed while timed, per_what)]; returns
    (rows, dominant row).  achieved = algorithmic flops (bytes) per item x
    items / total event time of the stage's launches."""
    rows = []
    for obj, items, per in owners:
        for i in range(obj.n_stages()):
            ms, cnt = obj.stage_time(i)
            if cnt == 0:
                continue
            name, fl, by = obj.stage_info(i)
            if name.startswith(("fe_", "sn_", "track")):
                b, pk, unit = stage_bound(name, precision)
            else:  # model stages: the same rule as the headline's stage table
                b, pk, unit = graph_stage_bound(name, fl, precision, by)
            work = (by * items / 1e9) if unit == "GB/s" else (fl * items / 1e12)
            a = work / (ms * 1e-3)
            rows.append({"kernel": name, "bound": b, "total_ms": round(ms, 4), "launches": cnt,
                         "ms_per_" + per: round(ms / max(items, 1) * (WINDOWS_PER_CLIP if per == "clip" else 1), 5),
                         "achieved": round(a, 2), "peak": pk, "unit": unit, "frac": round(a / pk, 4)})
    dom = max(rows, key=lambda r: r["total_ms"]) if rows else None
    return rows, dom


LINE_LIMIT = 8000  # the driver keeps ~8 KB of stdout: the whole line must fit (r05's 28.9 KB did not parse)
_ROOF_KEYS = ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic", "algorithmic_bytes",
              "algorithmic_flops", "avg_ms", "launches_timed", "overlapped_avg_ms", "traffic_source",
              "step_tflops", "whole_step", "anchor")
_SEC_KEYS = ("value", "ms_per_step", "dtype", "max_abs_dlogit", "frac", "gate")


def compact_line(out, full_path=None):
    """The one JSON line bench.py prints: the contract's fields, the dominant
    kernel's scalar roofline, cpu_baseline, the parity gate, and each
    secondary as {value, ms_per_step, dtype, max_abs_dlogit, frac} -- the
    per-stage tables go to ``full_path`` (the full record) instead.  Raises if
    the line would exceed LINE_LIMIT characters."""
    line = {k: v for k, v in out.items() if k not in ("roofline", "secondary", "config")}
    cfg = dict(out.get("config", {}))
    if isinstance(cfg.get("workload"), str):
        cfg["workload"] = cfg["workload"][:160]
    line["config"] = cfg
    if "roofline" in out:
        r = out["roofline"]
        line["roofline"] = {k: r[k] for k in _ROOF_KEYS if k in r}
    sec = {}
    for name, e in (out.get("secondary") or {}).items():
        s = {}
        for k in _SEC_KEYS:
            if k in e:
                s[k] = e[k]
        d = s.get("max_abs_dlogit")
        if isinstance(d, dict):  # main_step's {precision: delta} form
            s["max_abs_dlogit"] = next((v for v in d.values() if isinstance(v, float)), None)
        if "parity_gate" in e:
            s["gate"] = bool(e["parity_gate"].get("pass"))
        elif e.get("gated") is not None and isinstance(s.get("max_abs_dlogit"), float) and e.get("gated"):
            s["gate"] = s["max_abs_dlogit"] <= LOGIT_GATE
        r = e.get("roofline")
        if isinstance(r, dict):
            if "frac" in r:
                s["frac"] = r["frac"]
            elif "dominant_frac" in r:
                s["frac"] = r["dominant_frac"]
            if "kernel" in r or "dominant_kernel" in r:
                s["kernel"] = str(r.get("kernel", r.get("dominant_kernel")))[:48]
        for k in ("warm_same_run", "files_per_rank", "clips_per_rank"):
            if k in e:
                s[k] = e[k]
            elif k in e.get("config", {}):
                s[k] = e["config"][k]
        sec[name] = s
    if sec:
        line["secondary"] = sec
    if full_path:
        line["full_record"] = str(full_path)
    text = json.dumps(line, separators=(",", ":"))
    if len(text) > LINE_LIMIT:
        raise ValueError(f"bench line is {len(text)} characters (> {LINE_LIMIT})")
    return text


def emit_line(out):
    """Write the full record beside the run (gpurun_out/, the stage tables),
    then print the compact line -- the last thing on stdout."""
    full = ROOT / "gpurun_out" / "bench_full.json"
    try:
        full.parent.mkdir(exist_ok=True)
        full.write_text(json.dumps(out, indent=1))
        rel = full.relative_to(ROOT).as_posix()
    except OSError:
        rel = None
    print(compact_line(out, rel), flush=True)


def main_step(args, world, rank, dev, emit=True):
    from tools.make_models import make_model
    tmp = tempfile.mkdtemp(prefix="aa_bench_")
    fe_s = fe_settings(args.model)
    workload = WORKLOADS[args.model]
    first = make_batch(rank, fe_s)
    if args.model == "effnetv2":
        # BatchNorm statistics from the log-mels of the bench's own clips
        # (3 windows of another seed's batch, through the oracle front end)
        from oracle import fe_oracle
        from tools.make_models import make_graph
        cal_pcm, _, cal_views = make_batch(rank + 1000, fe_s)
        cfg = fe_config(fe_s)
        calib = np.stack([fe_oracle.window_logmel(window_samples(cal_pcm, v, cfg["win_len"]), cfg)
                          for v in cal_views[::len(cal_views) // 3][:3]])
        model_path = make_graph(Path(tmp) / "effnetv2", "effnetv2", in_channels=3, T=fe_s.n_frames, seed=5,
                                calib=calib)
    else:
        model_path = make_model(Path(tmp) / "model1", "model1", seed=1)
    pcm_np, _, views = first
    step = Step(dev, rank, model_path, args.precision, pairs=HEAD_PAIRS, first=first, lm16=args.logmel == "f16",
                pipeline=args.pipeline, fe_s=fe_s)
    fe, model, n_win = step.fe, step.model, step.n_win

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # calibration (untimed): one pass with every launch bracketed finds the
    # stages that launch (a fused stage launches nothing); then each stage is
    # timed on its own -- events around that launch only, 5 steps each -- so no
    # stage pays for its neighbours' events (bracketing them all inflates the
    # sum past the step).  The dominant stage gets the events of the timed region.
    # (the calibration runs serially: with the pipeline on, a stage's events
    # would also time whatever of the other stream overlaps it)
    pipelined, step.pipeline = step.pipeline, False
    lanes, step.lanes = step.lanes, None
    fe.set_timing(True)
    model.set_timing(True)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    launched = [c for c in collect(step.launches(), n_win) if c["count"] > 0]
    fe.set_timing(False)
    model.set_timing(False)
    launches = [(c["owner"], c["idx"]) for c in launched]
    calib = []
    for owner, idx in launches:
        owner.set_timing(True, stages=[idx])
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        calib.append(collect([(owner, idx)], n_win)[0])
        owner.set_timing(False)
    step.pipeline, step.lanes = pipelined, lanes
    step.k, step.issued = 0, -1
    seen_names = {}
    for c in calib:  # a graph repeats kernel shapes: stage names made unique
        k = seen_names.get(c["name"], 0)
        seen_names[c["name"]] = k + 1
        if k:
            c["name"] = f"{c['name']}#{k}"
    dom = max(calib, key=lambda x: x["avg_ms"])
    # the dominant kernel's roofline: HIP events around its launches over a
    # timed run of the SERIAL step (K steps, back to back on one stream: the
    # kernel alone on the GPU, what rocprofv3's kernel trace of the serial
    # step shows); then the headline timed region, overlapped, with events
    # around the same launches (there they also count the wait behind the
    # other stream's kernels)
    dom["owner"].set_timing(True, stages=[dom["idx"]])
    if pipelined or lanes is not None:
        step.pipeline, step.lanes = False, None
        timed(step, args.steps, 2, world)
        dom_serial = collect([(dom["owner"], dom["idx"])], n_win)[0]
        step.pipeline, step.lanes = pipelined, lanes
        step.k, step.issued = 0, -1
    elapsed = timed(step, args.steps, 2 if (pipelined or lanes is not None) else 0, world)
    dom_live = collect([(dom["owner"], dom["idx"])], n_win)[0]
    if not (pipelined or lanes is not None):
        dom_serial = dom_live
    dom["owner"].set_timing(False)
    # collectives on the device over RCCL; on the host when ranks share a GPU (gloo)
    cdev = dev if (world > 1 and dist.get_backend() == "nccl") else torch.device("cpu")
    ppg = max(1, args.procs_per_gpu) if args.config in (2, 4) else 1  # as worker() places ranks
    t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        # the per-file result gather (§8e): every rank's per-track records to all
        from aa_amd import shard
        rec = torch.from_numpy(shard.pack_records([2 * rank, 2 * rank + 1], [0, 0], step.tmean.cpu().numpy(),
                                                  width=model.n_labels)).to(cdev)
        gathered = shard.gather_records(rec)
        assert gathered.shape[0] == 2 * world
    elapsed = float(t.item())

    is_fe = dom["owner"] is fe
    if is_fe and dom["name"].startswith("fe_stft"):
        bound, peak, unit = "valu", VALU_F32_PEAK, "TFLOP/s"
    elif is_fe:
        bound, peak, unit = "hbm", HBM_PEAK_GBS, "GB/s"
    else:
        bound, peak, unit = graph_stage_bound(dom["name"], dom["flops"], args.precision, dom["bytes"])
    avg_s = dom_serial["avg_ms"] * 1e-3
    achieved = (dom["bytes"] / avg_s / 1e9) if unit == "GB/s" else (dom["flops"] / avg_s / 1e12)
    traffic, traffic_src = None, None
    tr, tr_path = load_traffic(len(launches) + 1, args.precision, workload)  # + track_mean
    if tr is not None:
        traffic = tr["kernels"][launches.index((dom["owner"], dom["idx"]))]["hbm_bytes"]
        traffic_src = tr_path
    roofline = {"bound": bound, "kernel": dom["name"], "achieved": round(achieved, 2), "peak": round(peak, 2),
                "unit": unit, "frac": round(achieved / peak, 4), "traffic": traffic,
                "algorithmic_bytes": round(dom["bytes"]), "algorithmic_flops": round(dom["flops"]),
                "avg_ms": round(dom_serial["avg_ms"], 4), "launches_timed": dom_serial["count"],
                "timed_on": "the serial step (K steps, one stream), events around this kernel's launches",
                "overlapped_avg_ms": round(dom_live["avg_ms"], 4),
                "traffic_source": traffic_src,
                "stages_ms": {c["name"]: round(c["avg_ms"], 4) for c in calib},
                "stages_sum_ms": round(sum(c["avg_ms"] for c in calib), 4)}
    # an in-run anchor: an HBM-streaming kernel whose code has not changed
    # since round 3 (fe_stats), timed in the same calibration pass, so a kernel
    # time compared across rounds (boxes differ by ~5 %) can be read as a ratio
    anc = next((c for c in calib if c["name"] == "fe_stats"), None)
    if anc is not None and anc["avg_ms"] > 0:
        roofline["anchor"] = {"kernel": "fe_stats", "avg_ms": round(anc["avg_ms"], 5),
                              "dominant_over_anchor": round(dom["avg_ms"] / anc["avg_ms"], 3),
                              "step_over_anchor": round((elapsed / args.steps * 1e3) / anc["avg_ms"], 2)}
    # every stage against its own bound (the dominant one above): algorithmic
    # flops or bytes of the calibration pass / its event-timed average
    per = {}
    for c in calib:
        fe_stage = c["owner"] is fe
        if fe_stage and c["name"].startswith("fe_stft"):
            b, pk, a = "valu", VALU_F32_PEAK, c["flops"] / (c["avg_ms"] * 1e-3) / 1e12
        elif fe_stage or c["flops"] == 0 or c["name"].startswith("head"):
            b, pk, a = "hbm", HBM_PEAK_GBS, c["bytes"] / (c["avg_ms"] * 1e-3) / 1e9
        else:
            b, pk, unit_c = graph_stage_bound(c["name"], c["flops"], args.precision, c["bytes"])
            a = (c["bytes"] / (c["avg_ms"] * 1e-3) / 1e9) if unit_c == "GB/s" else \
                c["flops"] / (c["avg_ms"] * 1e-3) / 1e12
        per[c["name"]] = {"bound": b, "achieved": round(a, 1), "frac": round(a / pk, 4)}
    roofline["stages"] = per
    # the same stages from a profile pass: rocprofv3's kernel trace of the
    # serial step (committed summary), kernels matched to launches in dispatch
    # order through the PMC summary's kernel names
    prof = load_profiled_stages(tr, args.precision)
    if prof is not None:
        stats_path, durs = prof
        ps = {}
        for c, us in zip(calib, durs):
            b = per[c["name"]]["bound"]
            pk = {"valu": VALU_F32_PEAK, "hbm": HBM_PEAK_GBS}.get(b, PEAK[args.precision])
            a = c["bytes"] / (us * 1e-6) / 1e9 if b == "hbm" else c["flops"] / (us * 1e-6) / 1e12
            ps[c["name"]] = {"bound": b, "avg_us": round(us, 2), "achieved": round(a, 1), "frac": round(a / pk, 4)}
        roofline["stages_profiled"] = ps
        roofline["stages_profiled_source"] = stats_path
    # whole step against the CNN's matrix roofline + the front end's VALU one
    step_flops = sum(c["flops"] for c in calib)
    roofline["step_tflops"] = round(step_flops / (elapsed / args.steps) / 1e12, 2)
    # the whole step against its ceiling (a graph model spreads its time over
    # ~100 stages, so no single kernel dominates it): every stage at the peak
    # of what binds it -- max(its FLOPs at its compute peak, its algorithmic
    # bytes at 8 TB/s), the compute peak being the FP32 VALU one for the FFT
    # and the exact-f32 graph convs, the precision's matrix peak for the MFMA
    # convs -- summed over the step's launches; compute_ceiling_ms keeps the
    # FLOPs-only figure (CNN at the matrix peak + front end at the VALU peak)
    fe_flops = sum(c["flops"] for c in calib if c["owner"] is fe)
    ceil_compute = (step_flops - fe_flops) / (PEAK[args.precision] * 1e12) + fe_flops / (VALU_F32_PEAK * 1e12)
    ceil_s = 0.0
    for c in calib:
        b = per[c["name"]]["bound"]
        pk = VALU_F32_PEAK if (b == "valu" or c["name"].startswith(("fe_stft", "conv_gf32"))) else PEAK[args.precision]
        ceil_s += max(c["flops"] / (pk * 1e12), c["bytes"] / (HBM_PEAK_GBS * 1e9))
    roofline["whole_step"] = {"bound": "per stage: mfma | valu | hbm", "step_gflop": round(step_flops / 1e9, 2),
                              "ceiling_ms": round(ceil_s * 1e3, 4), "compute_ceiling_ms": round(ceil_compute * 1e3, 4),
                              "achieved_tflops": roofline["step_tflops"], "peak_tflops": PEAK[args.precision],
                              "frac_of_matrix_peak": round(roofline["step_tflops"] / PEAK[args.precision], 4),
                              "frac_of_ceiling": round(ceil_s / (elapsed / args.steps), 4)}

    audio_s = world * args.steps * n_win * SECONDS_PER_WINDOW
    out = {
        "metric": METRIC, "value": round(audio_s / elapsed, 1), "unit": "audio-s/s", "n_gpus": max(1, world // ppg),
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None,
        "dtype": args.precision + (" (fp16 log-mel)" if args.logmel == "f16" else ""),
        "data": f"synthetic (48 kHz int16-quantised noise+chirps, seeded), seeded random-init {args.model}",
        "config": {"workload": workload, "model": args.model, "global_batch": n_win * world,
                   "seq_len": step.fe_s.win_len, "parallelism": f"dp{world}",
                   "pipeline": f"{len(step.lanes)} batches in flight on {len(step.lanes)} streams"
                               if step.lanes is not None else
                               "front end of batch k+1 on a second stream beside the CNN of batch k"
                               if step.pipeline else "serial",
                   "clip_pairs": f"{HEAD_PAIRS} resident clip pairs in rotation, one per step"},
        "roofline": roofline,
    }
    gate_fail = None
    cfg = fe_config(step.fe_s)
    ref = None
    if not args.no_parity:
        # every rank checks its own pair 0 (its clips differ per rank) against
        # the oracle, after the timed region; the worst delta over the ranks is
        # the line's, so an N-GPU line carries throughput only with parity
        # asserted on every GPU
        if world > 1:
            torch.set_num_threads(max(1, min(16, (os.cpu_count() or 8) // world)))
        ref = reference_logits(pcm_np, views, model_path, cfg)
        step.k, step.issued = 0, -1  # one more step on pair 0, the one the oracle ran
        step()
        torch.cuda.synchronize()
        d = float(np.abs(step.logits.cpu().numpy() - ref).max())
        if world > 1:
            dt = torch.tensor([d], dtype=torch.float64, device=cdev)
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
            d = float(dt.item())
        out["max_abs_dlogit"] = {args.precision: d}
        if world > 1:
            out["max_abs_dlogit"]["over"] = f"max over {world} ranks, each on its own clip pair"
        if args.precision in GATED:
            out["parity_gate"] = {"tol": LOGIT_GATE, "pass": d <= LOGIT_GATE, "ranks_checked": world}
            if d > LOGIT_GATE:
                gate_fail = f"{args.precision}: max|dlogit| {d:.3e} > {LOGIT_GATE}"
    if rank == 0 and world == 1:
        sec = {}
        modes = [m for m in args.secondary.split(",") if m]
        if args.model != "model1":  # the other workloads are model1's
            modes = [m for m in modes if m in ("serial", "f32")]
        if "effnetv2" in modes:
            # the efficientnet route (src/identify_tracks.py:539-540) as its own
            # bounded, gated run of this same function: EfficientNetV2-B0-shaped
            # graph, 3-channel log-mel at hop 281
            a2 = argparse.Namespace(**vars(args))
            a2.model, a2.secondary, a2.cpu_seconds, a2.steps = "effnetv2", "", 0, max(10, args.steps // 2)
            e = main_step(a2, 1, rank, dev, emit=False)
            sec["effnetv2"] = {k: e[k] for k in ("value", "ms_per_step", "steps", "dtype", "config", "max_abs_dlogit",
                                                 "parity_gate") if k in e}
            r = e["roofline"]
            sec["effnetv2"]["roofline"] = dict(r["whole_step"], dominant_kernel=r["kernel"],
                                               dominant_frac=r["frac"], stages_sum_ms=r["stages_sum_ms"],
                                               stages_ms=r["stages_ms"], stages=r["stages"])
            modes.remove("effnetv2")
        for mode in [m for m in modes if m.startswith("config")]:
            # BASELINE configs[2] / configs[3] as bounded runs on this GPU, each
            # with the roofline of its own dominant kernel
            if mode == "config3":
                sec[mode] = run_stream(args, 1, rank, dev, clips=args.clips, roofline=True)
            elif mode == "config4":
                sec[mode] = run_corpus(args, 1, rank, dev, files=args.files, roofline=True)
        for mode in [m for m in modes if not m.startswith("config")]:
            # "fp8_f16mel": BASELINE configs[4] (fp16 log-mel + fp8 CNN)
            prec = args.precision if mode in ("cold", "serial") else mode.split("_")[0]
            if mode == args.precision:
                continue
            pairs = COLD_POOL if mode == "cold" else int(mode[4:]) if mode.startswith("pool") else HEAD_PAIRS
            if mode.startswith("pool"):
                prec = args.precision
            s2 = Step(dev, rank, model_path, prec, pairs=pairs, first=first,
                      lm16=mode.endswith("_f16mel") or (mode in ("cold", "serial") and args.logmel == "f16"),
                      pipeline=0 if mode == "serial" else args.pipeline, fe_s=fe_s)
            n2 = args.steps if mode in ("cold", "serial") or mode.startswith("pool") else max(10, args.steps // 2)
            if mode == "cold":
                # cold and the headline step alternated three times, medians:
                # box clocks drift by several % between back-to-back runs
                els, elw = [], []
                for _ in range(3):
                    els.append(timed(s2, n2, 5, 1))
                    elw.append(timed(step, n2, 5, 1))
                el, el_w = sorted(els)[1], sorted(elw)[1]
            else:
                el = timed(s2, n2, 5, 1)
            e = {"value": round(n2 * s2.n_win * SECONDS_PER_WINDOW / el, 1), "ms_per_step": round(1e3 * el / n2, 4),
                 "steps": n2, "dtype": prec + (" (fp16 log-mel)" if s2.logmel.dtype == torch.float16 else "")}
            e["pipeline"] = len(s2.lanes) if s2.lanes is not None else int(s2.pipeline)
            if mode == "serial":
                e["note"] = "front end and CNN back to back on one stream (no overlap across steps)"
            if mode == "cold":
                e["note"] = f"fresh clip pair per step from {COLD_POOL} resident pairs (> Infinity Cache)"
                e["warm_same_run"] = round(n2 * n_win * SECONDS_PER_WINDOW / el_w, 1)
                e["cold_over_warm"] = round(el_w / el, 4)
            if mode.startswith("pool"):
                e["note"] = f"{pairs} resident clip pairs in rotation (inside the Infinity Cache)"
            if mode.startswith("fp8"):
                # configs[4]'s kernels against their own bounds: events around
                # every launch of 5 serial steps (untimed for the value above)
                pl, ln = s2.pipeline, s2.lanes
                s2.pipeline, s2.lanes = False, None
                for o in (s2.fe, s2.model):
                    o.set_timing(True)
                for _ in range(5):
                    s2()
                torch.cuda.synchronize()
                for o in (s2.fe, s2.model):
                    o.set_timing(False)
                s2.pipeline, s2.lanes = pl, ln
                rows, dom = stage_table([(s2.fe, 5 * s2.n_win, "window"), (s2.model, 5 * s2.n_win, "window")], prec)
                e["roofline"] = dict(dom, timed_on="HIP events around every launch of 5 serial steps", stages=rows)
            if mode != "cold" and not mode.startswith("pool") and ref is not None:
                s2.k, s2.issued = 0, -1
                s2()
                torch.cuda.synchronize()
                e["max_abs_dlogit"] = float(np.abs(s2.logits.cpu().numpy() - ref).max())
                e["gated"] = prec in GATED
            sec[mode] = e
            del s2
        if sec:
            out["secondary"] = sec
        if args.cpu_seconds > 0:
            v, nw, dt = cpu_baseline(pcm_np, views, model_path, cfg, args.cpu_seconds, args.cpu_workers)
            out["cpu_baseline"] = {"value": round(v, 2), "unit": "audio-s/s", "cores": args.cpu_workers,
                                   "kind": "port",
                                   "sample": f"{nw} windows (the step's 64, cycled; oracle numpy FE on "
                                             f"{args.cpu_workers} processes + torch-CPU fp32 {args.model} on "
                                             f"{args.cpu_workers} threads), {dt:.1f} s"}
        # a gated secondary (the f32 step, the efficientnet route) that misses
        # the 1e-3 gate fails the bench like the headline does
        bad = [m for m, e in sec.items()
               if (e.get("parity_gate") is not None and not e["parity_gate"].get("pass"))
               or (e.get("gated") and e.get("max_abs_dlogit", 0.0) > LOGIT_GATE)]
        if bad and not gate_fail:
            gate_fail = "secondary " + ", ".join(bad) + f": max|dlogit| > {LOGIT_GATE}"
    if not emit:
        return out  # (a secondary: its parity_gate entry carries the verdict)
    if rank == 0:
        emit_line(out)
    if gate_fail:
        raise SystemExit(f"parity gate failed: {gate_fail}")
    return out


def main_stream(args, world, rank, dev):
    out = run_stream(args, world, rank, dev)
    if rank == 0:
        emit_line(out)


def run_stream(args, world, rank, dev, clips=None, roofline=False):
    """configs[2]: clips streamed through aa_amd.stream.StreamRunner (host PCM
    -> pinned staging -> copy stream, double-buffered against the kernels),
    model1+model2+model3 sharing one front end; one 0-60 s track per clip
    (39 windows).  value = clips x 60 s over all ranks / max-over-ranks wall
    time, host->device transfer included.  With N ranks every rank streams its
    own clips and the per-track scores are all-gathered (RCCL) at the end."""
    from aa_amd import shard
    from aa_amd.stream import Recording, StreamRunner
    from tools import synth
    from tools.make_models import make_ensemble

    class Track:
        start, end, freq_start, freq_end, length = 0.0, 60.0, 0, 24000, 60.0

    fe_s = fe_settings()
    root = Path(tempfile.mkdtemp(prefix="aa_bench3_"))
    make_ensemble(root)
    paths = [root / m / "audioModel.safetensors" for m in ("model1", "model2", "model3")]
    pool = [synth.clip(1000 * rank + i) for i in range(8)]  # distinct PCM, cycled (host synthesis untimed)
    runner = StreamRunner(paths, fe_s, precision=args.precision, device=dev, max_windows=8 * WINDOWS_PER_CLIP,
                          max_samples=8 * len(pool[0]))

    def clip_iter(n, first=0):
        return (Recording(key=first + i, pcm=pool[i % len(pool)], tracks=[Track()]) for i in range(n))

    n_clips = int(clips or args.clips)
    for _ in runner.run(clip_iter(32)):
        pass
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    results = list(runner.run(clip_iter(n_clips, first=rank * n_clips)))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    assert len(results) == n_clips
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    n_gathered = len(results)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        rec = shard.pack_records([k for k, _, _ in results], [ti for _, ti, _ in results],
                                 np.stack([s for _, _, s in results]), width=runner.L)
        n_gathered = int(shard.gather_records(torch.from_numpy(rec).to(dev)).shape[0])
        assert n_gathered == world * n_clips
    elapsed = float(t.item())
    out = {"metric": METRIC, "value": round(world * n_clips * 60.0 / elapsed, 1), "unit": "audio-s/s",
           "n_gpus": world, "steps": n_clips, "warmup": 32,
           "ms_per_step": round(1e3 * elapsed / n_clips, 4), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": args.precision,
           "data": "synthetic (48 kHz int16-quantised noise+chirps, seeded), seeded random-init model1/2/3",
           "config": {"workload": "config3: 60 s clips streamed from host memory, 39 windows each, "
                                  "model1+model2+model3 ensemble, 8 clips per batch",
                      "model": "model1+model2+model3", "global_batch": 8 * WINDOWS_PER_CLIP * world,
                      "seq_len": fe_s.win_len, "parallelism": f"dp{world}", "clips_per_rank": n_clips,
                      "records_gathered": n_gathered}}
    if roofline:
        # the stream's kernels, HIP events around every launch over 16 more
        # clips (untimed for the value above)
        objs = [runner.fe] + list(runner.models)
        for o in objs:
            o.set_timing(True)
        list(runner.run(clip_iter(16)))
        torch.cuda.synchronize()
        for o in objs:
            o.set_timing(False)
        rows, dom = stage_table([(o, 16 * WINDOWS_PER_CLIP, "clip") for o in objs], args.precision)
        out["roofline"] = dict(dom, timed_on="HIP events around every launch of 16 streamed clips",
                               stages=rows)
    return out


def _write_clip(path, seed):
    from tools import synth
    synth.write_wav(path, synth.clip(seed))


def main_corpus(args, world, rank, dev):
    out = run_corpus(args, world, rank, dev)
    if rank == 0:
        emit_line(out)


def run_corpus(args, world, rank, dev, files=None, roofline=False):
    """configs[3]: a corpus of 60 s WAV files through the whole analyse path
    (aa_amd.corpus: decode, signal_noise, tracks, classify() with model1,
    post-processing to the reference's per-file JSON), files sharded one per
    stream across ranks and the JSON documents all-gathered (RCCL) at the end.
    value = files x 60 s over all ranks / max-over-ranks wall time, including
    the file reads and the host-side steps the reference runs on the CPU."""
    from aa_amd import corpus
    from tools import synth
    from tools.make_models import make_model
    root = Path(tempfile.mkdtemp(prefix="aa_bench4_"))
    model = make_model(root / "model1", "model1", seed=1)
    n = int(files or args.files)
    # a pool of CORPUS_POOL distinct WAVs per rank, cycled to n files per rank
    # (the file list repeats paths; every entry is decoded and analysed anew,
    # from the page cache): configs[3]'s 1,250 files per GPU without writing
    # 7 GB of WAVs first
    n_pool = min(n, CORPUS_POOL) * world
    files = [root / f"clip{i % n_pool:05d}.wav" for i in range(n * world)]
    # every rank writes its own share of the pool (plus file 0 for the
    # warm-up) into its own temp dir, on a pool of host processes
    mine = [i for i in range(n_pool) if i % world == rank or i == 0]
    from concurrent.futures import ProcessPoolExecutor
    import multiprocessing as mpc
    with ProcessPoolExecutor(max_workers=min(16, len(mine)), mp_context=mpc.get_context("spawn")) as ex:
        list(ex.map(_write_clip, [str(files[i]) for i in mine], [5000 + i for i in mine]))
    models = [str(model)]
    ppg = max(1, args.procs_per_gpu)
    cdev = dev if (world > 1 and dist.get_backend() == "nccl") else torch.device("cpu")  # collectives
    n_gpus = max(1, world // ppg)
    # warm-up (untimed): plans, kernels, model upload, and every pinned staging
    # slot the timed run holds (aa_amd.batch: (lanes + PREFETCH) batches; a slot pool
    # grown inside the timed run allocated ~6 MB of pinned memory per slot there)
    from aa_amd import batch as _batch
    lanes = corpus.default_lanes()
    corpus.run([files[0]] * (max(4, lanes + _batch.PREFETCH) * max(args.batch, 1)), models, rank=0, world=1,
               batch=args.batch)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    res = corpus.run(files, models, rank=rank, world=world, device=cdev if world > 1 else None, batch=args.batch)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    assert len(res) == n * world
    failed = [i for i, r in res.items() if corpus.failed(r)]
    assert not failed, f"corpus files failed: {failed[:4]}"
    t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    n_pred = sum(len(r.get("species_identify", [])) for r in res.values())
    out = {"metric": METRIC, "value": round(n * world * 60.0 / elapsed, 1), "unit": "audio-s/s", "n_gpus": n_gpus,
           "steps": n, "warmup": 1, "ms_per_step": round(1e3 * elapsed / n, 4), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "bf16x3",
           "data": "synthetic 60 s 48 kHz int16 WAV files (noise+chirps, seeded), seeded random-init model1",
           "config": {"workload": "config4: corpus of 60 s WAV files through analyse.examine (decode, "
                                  "signal_noise, tracks, classify, species JSON), files sharded over ranks, K per device pass, "
                                  "JSON all-gathered", "model": "model1", "global_batch": world * max(args.batch, 1),
                      "files_per_device_pass": max(args.batch, 1),
                      "seq_len": 48000 * 60, "parallelism": f"dp{n_gpus}", "host_procs_per_gpu": ppg,
                      "files_per_rank": n, "distinct_wavs_per_rank": n_pool // world,
                      "documents_gathered": len(res), "tracks_classified": n_pred}}
    if roofline:
        # the corpus path's kernels (signal_noise, get_end, front end, CNN),
        # HIP events around every launch over 32 more files (untimed above)
        from aa_amd.pipeline import Classifier
        from aa_amd.signals import detector
        clf = Classifier.shared(device=dev)
        det = detector(48000, 281, dev)
        fes, mods = list(clf._fes.values()), list(clf._models.values())
        objs = [det] + fes + mods
        for o in objs:
            o.set_timing(True)
        w0 = clf.windows_done
        sub = files[:32]
        lanes_env = os.environ.get("AA_BATCH_LANES")
        os.environ["AA_BATCH_LANES"] = "1"  # one host thread: the stage timers are not shared across lanes
        try:
            corpus.run(sub, models, rank=0, world=1, batch=args.batch)
            torch.cuda.synchronize()
        finally:
            if lanes_env is None:
                os.environ.pop("AA_BATCH_LANES")
            else:
                os.environ["AA_BATCH_LANES"] = lanes_env
        for o in objs:
            o.set_timing(False)
        wins = clf.windows_done - w0
        frames = len(sub) * det.n_frames(48000 * 60)
        rows, dom = stage_table([(det, frames, "frame")] + [(o, wins, "window") for o in fes + mods], "bf16x3")
        per_file = {r["kernel"]: round(r["total_ms"] / len(sub), 4) for r in rows}
        out["roofline"] = dict(dom, timed_on=f"HIP events around every launch of {len(sub)} corpus files "
                                             f"({frames} signal_noise frames, {wins} windows)",
                               ms_per_file=per_file, stages=rows)
    import shutil
    shutil.rmtree(root, ignore_errors=True)  # (5.8 MB per file)
    return out


def worker(local, world, args, port=None):
    """One rank.  ``port`` set: spawned by ``--gpus N`` (no torchrun env)."""
    if port is not None:
        os.environ.update(RANK=str(local), LOCAL_RANK=str(local), WORLD_SIZE=str(world),
                          MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    rank = int(os.environ.get("RANK", "0"))
    ppg = max(1, args.procs_per_gpu) if args.config in (2, 4) else 1
    gpu = local // ppg
    if world > 1:
        if ppg > 1:  # ranks sharing a GPU: RCCL needs one rank per device
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    from aa_amd import _lib
    _lib.lib()  # fails loudly without the HIP library
    try:
        if args.config == 3:
            main_stream(args, world, rank, dev)
        elif args.config == 4:
            main_corpus(args, world, rank, dev)
        else:
            main_step(args, world, rank, dev)
    finally:
        if world > 1:
            dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main(argv=None):
    args = parse(argv)
    if "WORLD_SIZE" in os.environ:  # torchrun: one process per GPU already
        worker(int(os.environ.get("LOCAL_RANK", "0")), int(os.environ["WORLD_SIZE"]), args)
    elif args.gpus > 1 or (args.config in (2, 4) and args.procs_per_gpu > 1):
        # spawn the ranks before this process touches the GPU
        import torch.multiprocessing as mp
        n = args.gpus * (max(1, args.procs_per_gpu) if args.config in (2, 4) else 1)
        mp.spawn(worker, args=(n, args, _free_port()), nprocs=n, join=True)
    else:
        worker(0, 1, args)


if __name__ == "__main__":
    main()
