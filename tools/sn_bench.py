"""Time signal_noise (aa_sn_run) on synthetic 60 s clips: wall time per clip
and, under rocprofv3 --kernel-trace --stats, the per-kernel split."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "audio-analysis_amd")]

import numpy as np
import torch

from aa_amd.signals import SignalDetector
from tools import synth


def main(n=50):
    dev = torch.device("cuda")
    det = SignalDetector(48000, 281, dev)
    clips = [torch.from_numpy(synth.clip(i)).to(dev) for i in range(4)]
    for c in clips:
        det.components(c)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    k = 0
    for i in range(n):
        # components() copies the count/status back: a host sync per clip, as classify() does
        det.components(clips[i % len(clips)])
        k += 1
    dt = (time.perf_counter() - t0) / k
    print(f"signal_noise 60 s clip: {dt * 1e3:.3f} ms/clip, {60.0 / dt:.0f} audio-s/s, "
          f"{len(det.components(clips[0]))} components in clip 0")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 50)
