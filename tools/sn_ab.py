"""signal_noise of the working-tree library against another build (AA_LIB,
e.g. tools/ablib/libaa_base.so from tools/ab_head.py): masks before morphology
and the component tables must be bit-identical; wall time per 60 s clip.

usage: python tools/sn_ab.py OUT.npz           (run once per library)
       python tools/sn_ab.py --compare A.npz B.npz"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "audio-analysis_amd")]

import numpy as np


def run(out):
    import torch
    from aa_amd.signals import SignalDetector
    from tools import synth
    dev = torch.device("cuda")
    det = SignalDetector(48000, 281, dev)
    res = {}
    lens = [2_880_000, 2_880_000 - 281 * 37 - 5, 3_600_000, 123_457, 281 * 64, 48000 * 75]
    for i, n in enumerate(lens):
        x = synth.clip(100 + i)
        x = np.resize(x, n).astype(np.float32)
        pcm = torch.from_numpy(x).to(dev)
        F = det.n_frames(n)
        mask = torch.zeros((2049, det.words(F)), dtype=torch.int64, device=dev)
        comp = det.components(pcm, mask_out=mask)
        res[f"mask{i}"] = mask.cpu().numpy()
        res[f"comp{i}"] = np.asarray(comp)
    clips = [torch.from_numpy(synth.clip(i)).to(dev) for i in range(4)]
    for c in clips:
        det.components(c)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(60):
        det.components(clips[i % 4])
    dt = (time.perf_counter() - t0) / 60
    res["ms_per_clip"] = np.float64(dt * 1e3)
    np.savez(out, **res)
    print(f"{out}: signal_noise 60 s clip {dt * 1e3:.3f} ms/clip")


def compare(a, b):
    A, B = np.load(a), np.load(b)
    bad = [k for k in A.files if k != "ms_per_clip" and not np.array_equal(A[k], B[k])]
    print(f"{a} {float(A['ms_per_clip']):.3f} ms vs {b} {float(B['ms_per_clip']):.3f} ms; "
          f"{len(A.files) - 1 - len(bad)} arrays equal, differing: {bad}")
    return 1 if bad else 0


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(compare(sys.argv[2], sys.argv[3]))
    run(sys.argv[1])
