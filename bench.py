"""Throughput benchmark of the MI355X hot path (BASELINE.json metric).

Workload (BASELINE.json configs[1], "config 2"): one step = one batch of 64
analysis windows -- 39 windows of a 60 s clip + 25 windows of a second 60 s
clip (48 kHz mono, synthetic, int16-quantised; reference stride 1.5 s / length
3 s) -- through the GPU log-mel front end (htk custom mel, n_fft 4096, hop 640,
160 bands, power_to_db) and the model1 CNN in bf16, then the per-track mean.
PCM and window tables are resident in HBM before the timed region.

Audio-seconds per step: a 60 s clip is covered by 39 windows, so each window
counts 60/39 s; value = (windows processed by all ranks x 60/39) / max-over-
ranks wall time.  Multi-GPU: one process per GPU, each with its own clips
(weak scaling); the only collective is the final RCCL gather of per-track
results (outside the per-step path, like the per-file result gather of §8e).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
from pathlib import Path

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
PEAK = {"bf16": 2500.0, "f32": 157.3}  # dense TFLOP/s, MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="bound on the CPU-baseline sample (0 disables)")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--streams", type=int, default=1,
                    help="split the step's windows over this many HIP streams (overlaps kernel tails)")
    return ap.parse_args()


def make_batch(rank, fe_settings):
    """Two resident 60 s clips and the 64-window table (39 + 25)."""
    from aa_amd.frontend import pack_windows
    from aa_amd.windows import track_windows
    from tools import synth
    a, b = synth.clip(2 * rank), synth.clip(2 * rank + 1)
    pcm = np.concatenate([a, b])
    sr = fe_settings.sr
    va = track_windows(len(a), sr, 0.0, 60.0, 60.0, 0, 24000, 3, 1.5, 50, 11000)
    vb = track_windows(len(b), sr, 0.0, 60.0, 60.0, 0, 24000, 3, 1.5, 50, 11000)[:BATCH_B]
    assert len(va) == BATCH_A
    rows = np.concatenate([pack_windows(va, len(a)), pack_windows(vb, len(b), offset=len(a))])
    views = [(s, n, p) for (s, n, p) in va] + [(s + len(a), n, p) for (s, n, p) in vb]
    return pcm, rows, views


def cpu_baseline(pcm, views, model_path, fe_cfg, budget_s):
    """Oracle (numpy librosa-0.11 restatement + torch-CPU fp32 CNN) on a bounded
    sample of the same windows; returns (audio-s/s, windows, seconds, logits)."""
    from oracle import cnn_oracle, fe_oracle
    threads = torch.get_num_threads()
    done, t0 = [], time.perf_counter()
    logits = []
    i = 0
    while i < len(views) and (time.perf_counter() - t0) < budget_s:
        chunk = views[i:i + 8]
        mels = []
        for (s, n, p) in chunk:
            w = np.zeros(fe_cfg["win_len"], np.float32)
            w[p:p + n] = pcm[s:s + n]
            mels.append(fe_oracle.window_logmel(w, fe_cfg))
        lg, _ = cnn_oracle.forward(model_path, np.stack(mels))
        logits.append(lg)
        done.extend(chunk)
        i += len(chunk)
    dt = time.perf_counter() - t0
    return len(done) * SECONDS_PER_WINDOW / dt, len(done), dt, threads, np.concatenate(logits)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from aa_amd import _lib
    from aa_amd.frontend import FeSettings, FrontEnd
    from aa_amd.model import Model, track_mean
    from tools.make_models import make_model

    _lib.lib()
    fe_s = FeSettings(htk=True, hop_length=640, n_fft=4096, n_mels=160, break_freq=1750)
    pcm_np, rows_np, views = make_batch(rank, fe_s)
    tmp = tempfile.mkdtemp(prefix="aa_bench_")
    model_path = make_model(Path(tmp) / "model1", "model1", seed=1)

    fe = FrontEnd(fe_s, dev)
    T = fe.T
    model = Model(model_path, (fe_s.n_mels, T, 1), precision=args.precision, device=dev)
    n_win = rows_np.shape[0]
    pcm = torch.from_numpy(pcm_np).to(dev)
    rows = torch.from_numpy(rows_np).to(dev)
    logmel = torch.empty(fe.out_shape(n_win), dtype=torch.float32, device=dev)
    logits = torch.empty((n_win, model.n_labels), dtype=torch.float32, device=dev)
    probs = torch.empty_like(logits)
    wb = torch.tensor([0, BATCH_A], dtype=torch.int32, device=dev)
    wc = torch.tensor([BATCH_A, BATCH_B], dtype=torch.int32, device=dev)
    tmean = torch.empty((2, model.n_labels), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream()
    # window chunks, one per stream, each with its own workspaces
    S = max(1, min(args.streams, n_win))
    bounds = np.linspace(0, n_win, S + 1).astype(int)
    chunks = [(int(a), int(b)) for a, b in zip(bounds[:-1], bounds[1:])]
    streams = [stream] if S == 1 else [torch.cuda.Stream(device=dev) for _ in range(S)]
    fe_ws = [torch.empty(max(fe.workspace_bytes(b - a), 256), dtype=torch.uint8, device=dev) for a, b in chunks]
    m_ws = [torch.empty(max(model.workspace_bytes(b - a), 256), dtype=torch.uint8, device=dev) for a, b in chunks]

    def run_chunks(fe_events=None):
        if S > 1:
            ev = torch.cuda.Event()
            ev.record(stream)
        for k, (a, b) in enumerate(chunks):
            s = streams[k]
            if S > 1:
                s.wait_event(ev)
            e0 = e1 = None
            if fe_events is not None and k == 0:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(s)
            fe.run(pcm, rows[a:b], out=logmel[a:b], stream=s, workspace=fe_ws[k])
            if e0 is not None:
                e1.record(s)
                fe_events.append((e0, e1, b - a))
            model.forward(logmel[a:b], logits[a:b], probs[a:b], stream=s, workspace=m_ws[k])
        if S > 1:
            for s in streams:
                done = torch.cuda.Event()
                done.record(s)
                stream.wait_event(done)
        track_mean(probs[None], wb, wc, out=tmean, stream=stream)

    def step():
        run_chunks()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # drop warmup timings, then time exactly K steps with per-stage events on
    model.set_timing(True)
    for i in range(model.n_stages()):
        model.stage_time(i)
    fe_ev = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run_chunks(fe_ev)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    model.set_timing(False)
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        # the per-file result gather (§8e): every rank's per-track records to all
        from aa_amd import shard
        rec = torch.from_numpy(shard.pack_records([2 * rank, 2 * rank + 1], [0, 0], tmean.cpu().numpy(),
                                                  width=model.n_labels)).to(dev)
        gathered = shard.gather_records(rec)
        assert gathered.shape[0] == 2 * world
    elapsed = float(t.item())

    stages = []
    for i in range(model.n_stages()):
        name, flops, byts = model.stage_info(i)
        ms, cnt = model.stage_time(i)
        # per launch: a launch covers one chunk of the step's windows
        per = n_win / S
        stages.append(dict(name=name, flops=flops * per, bytes=byts * per,
                           avg_ms=ms / max(cnt, 1), count=cnt))
    fe_ms = sum(a.elapsed_time(b) for a, b, _ in fe_ev) / max(len(fe_ev), 1)
    dom = max(stages, key=lambda s: s["avg_ms"])
    achieved = dom["flops"] / (dom["avg_ms"] * 1e-3) / 1e12
    roofline = {"bound": "mfma", "kernel": dom["name"], "achieved": round(achieved, 2),
                "peak": PEAK[args.precision], "unit": "TFLOP/s",
                "frac": round(achieved / PEAK[args.precision], 4), "traffic": None,
                "avg_ms": round(dom["avg_ms"], 4),
                "stages_ms": {s["name"]: round(s["avg_ms"], 4) for s in stages},
                "frontend_ms": round(fe_ms, 4)}

    audio_s = world * args.steps * n_win * SECONDS_PER_WINDOW
    value = audio_s / elapsed
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "audio-s/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
        "data": "synthetic (48 kHz int16-quantised noise+chirps, seeded), seeded random-init model1",
        "config": {"workload": "config2: 64 windows/step (39 of clip A + 25 of clip B, 60 s "
                               "48 kHz mono), htk log-mel n_fft 4096 hop 640 160 mel + model1 CNN",
                   "model": "model1", "global_batch": n_win * world, "seq_len": fe_s.win_len,
                   "parallelism": f"dp{world}", "streams": S},
        "roofline": roofline,
    }
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        fe_cfg = dict(sr=fe_s.sr, hop_length=fe_s.hop_length, n_mels=fe_s.n_mels, fmin=fe_s.fmin,
                      fmax=fe_s.fmax, n_fft=fe_s.n_fft, power=fe_s.power, db_scale=True, htk=True,
                      break_freq=fe_s.break_freq, normalize=True, win_len=fe_s.win_len)
        v, nw, dt, thr, ref_logits = cpu_baseline(pcm_np, views, model_path, fe_cfg, args.cpu_seconds)
        out["cpu_baseline"] = {"value": round(v, 2), "unit": "audio-s/s", "cores": thr,
                               "kind": "port",
                               "sample": f"{nw} of the step's 64 windows (oracle numpy FE + "
                                         f"torch-CPU fp32 model1), {dt:.1f} s"}
        if not args.no_parity:
            g = logits[:nw].cpu().numpy()
            out["max_abs_dlogit"] = {args.precision: float(np.abs(g - ref_logits).max())}
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
