"""Front-end micro-benchmark: time aa_fe_run variants with HIP events."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "audio-analysis_amd")]
import numpy as np
import torch

from aa_amd.frontend import FeSettings, FrontEnd, pack_windows
from aa_amd.windows import track_windows
from tools import synth


def run(settings, n_win, iters=20):
    clip = np.concatenate([synth.clip(0), synth.clip(1)])
    va = track_windows(2_880_000, 48000, 0.0, 60.0, 60.0, 0, 24000, 3, 1.5, 50, 11000)
    views = (va + [(s + 2_880_000, n, p) for s, n, p in va]) * ((n_win + 77) // 78)
    views = views[:n_win]
    fe = FrontEnd(settings)
    pcm = torch.from_numpy(clip).cuda()
    win = torch.from_numpy(pack_windows(views, len(clip))).cuda()
    out = torch.empty(fe.out_shape(n_win), device="cuda")
    for _ in range(3):
        fe.run(pcm, win, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fe.run(pcm, win, out=out)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


if __name__ == "__main__":
    for name, s in [("htk_norm", FeSettings(htk=True)),
                    ("htk_nonorm", FeSettings(htk=True, normalize=False)),
                    ("htk_nodb", FeSettings(htk=True, db_scale=False)),
                    ("hop281", FeSettings(htk=True, hop_length=281)),
                    ("nfft2048", FeSettings(htk=True, n_fft=2048))]:
        for n in (16, 64, 256):
            print(f"{name:12s} n_win={n:4d} {run(s, n):9.1f} us", flush=True)
