"""Host-side cost of the corpus path's host -> device copies (GPU box):
pinned-slot views copied with non_blocking, pageable numpy arrays through
.to(dev), and the pinned staging alternative, each while the stream is busy
with a long kernel (does the call return before the copy runs?).

    python tools/h2d_probe.py
"""
import time

import numpy as np
import torch


def busy(dev, ms=20.0):
    """Queue ~ms of device work on the current stream."""
    a = torch.randn(4096, 4096, device=dev)
    t0 = time.perf_counter()
    n = 0
    ev = torch.cuda.Event(enable_timing=True)
    e0 = torch.cuda.Event(enable_timing=True)
    e0.record()
    while True:
        a = a @ a
        a = a / a.norm()
        n += 1
        ev.record()
        ev.synchronize()
        if e0.elapsed_time(ev) > ms:
            break
    return n


def main():
    dev = torch.device("cuda")
    torch.cuda.init()
    x = torch.randn(4096, 4096, device=dev)
    for _ in range(3):  # warm up
        y = x @ x
    torch.cuda.synchronize()
    slot = torch.empty(6 << 20, dtype=torch.uint8, pin_memory=True)
    view = slot[44:44 + 5_760_000].view(torch.int16)
    dst = torch.empty(view.numel(), dtype=torch.int16, device=dev)
    small = np.arange(4096, dtype=np.int32)
    for label, fn in [
        ("pinned view copy_ non_blocking (5.76 MB)", lambda: dst.copy_(view, non_blocking=True)),
        ("pageable .to(dev) (16 KB)", lambda: torch.from_numpy(small).to(dev)),
        ("pinned staging .to(dev, non_blocking) (16 KB)",
         lambda: torch.from_numpy(small).pin_memory().to(dev, non_blocking=True)),
        ("pageable .cpu() of a 16 KB device tensor", lambda: dst[:8192].cpu()),
    ]:
        ts = []
        for _ in range(5):
            # a long chain of matmuls queued first: a synchronous call waits for it
            for _ in range(40):
                y = x @ x
            t0 = time.perf_counter()
            fn()
            ts.append(1e3 * (time.perf_counter() - t0))
            torch.cuda.synchronize()
        print(f"{label:50s} host ms per call: " + " ".join(f"{t:.2f}" for t in ts), flush=True)
    t0 = time.perf_counter()
    for _ in range(40):
        y = x @ x
    torch.cuda.synchronize()
    print(f"{'(the queued work alone)':50s} {1e3 * (time.perf_counter() - t0):.2f} ms")


if __name__ == "__main__":
    main()
