"""Time signal_noise on synthetic 60 s clips (through gpurun): wall time per
clip of aa_sn_run (one recording, host sync per clip as classify() does) and
of aa_sn_run_batch (K recordings per call, the corpus path), then every
launch stage's HIP-event time per clip against its roofline.  Under
rocprofv3 --kernel-trace --stats it gives the per-kernel split."""
import ctypes as C
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "audio-analysis_amd")]

import torch

from aa_amd import _lib
from aa_amd.signals import SignalDetector
from tools import synth


def main(n=40, K=8):
    import bench
    dev = torch.device("cuda")
    det = SignalDetector(48000, 281, dev)
    clips = [torch.from_numpy(synth.clip(i)).to(dev) for i in range(K)]
    for c in clips:
        det.components(c)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        det.components(clips[i % K])
    single = (time.perf_counter() - t0) / n
    # the batch form over K clips laid out in one buffer
    L = _lib.lib()
    pcm = torch.cat(clips)
    N = clips[0].numel()
    offs = (C.c_int64 * K)(*[k * N for k in range(K)])
    lens = (C.c_int64 * K)(*[N] * K)
    ws = torch.empty(L.aa_sn_batch_workspace_bytes(det._h, N, K), dtype=torch.uint8, device=dev)
    out = torch.zeros((K, 513, 6), dtype=torch.int32, device=dev)

    def batch():
        _lib.check(L.aa_sn_run_batch(det._h, _lib.dptr(pcm), offs, lens, K, _lib.dptr(ws), ws.numel(),
                                     _lib.dptr(out[0, 1:]), 512, 513, _lib.dptr(out[0, 0]), 513 * 6,
                                     _lib.stream_ptr()), "aa_sn_run_batch")

    batch()
    torch.cuda.synchronize()
    reps = max(2, n // K)
    t0 = time.perf_counter()
    for _ in range(reps):
        batch()
    torch.cuda.synchronize()
    batched = (time.perf_counter() - t0) / (reps * K)
    det.set_timing(True)
    for _ in range(2):
        batch()
    torch.cuda.synchronize()
    det.set_timing(False)
    rows, dom = bench.stage_table([(det, 2 * K * det.n_frames(N), "frame")], "bf16x3")
    for r in rows:
        r["ms_per_clip"] = round(r["total_ms"] / (2 * K), 4)
    print(json.dumps({"single_ms_per_clip": round(single * 1e3, 4), "batch_ms_per_clip": round(batched * 1e3, 4),
                      "batch_audio_s_per_s": round(60.0 / batched, 1), "K": K, "dominant": dom["kernel"],
                      "stages": rows}, indent=1))


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
