"""Host cost of aa_sn_run_batch's launches (through gpurun): the time the
ctypes call takes to return (its ~140 kernel launches for K = 32
recordings) against the device time of the batch, from one thread and from
T threads on streams of their own at once (the corpus lanes).

    python tools/sn_launch_probe.py [K] [T]
"""
import ctypes as C
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "audio-analysis_amd")]

import torch

from aa_amd import _lib
from aa_amd.signals import SignalDetector
from tools import synth


def main(K=32, T=8, reps=4):
    dev = torch.device("cuda", 0)
    L = _lib.lib()
    det = SignalDetector(48000, 281, dev)
    base = [torch.from_numpy(synth.clip(i)).to(dev) for i in range(4)]
    N = base[0].numel()
    pcm = torch.cat([base[k % 4] for k in range(K)])
    offs = (C.c_int64 * K)(*[k * N for k in range(K)])
    lens = (C.c_int64 * K)(*[N] * K)
    need = L.aa_sn_batch_workspace_bytes(det._h, N, K)

    class Lane:
        def __init__(self):
            self.ws = torch.empty(need, dtype=torch.uint8, device=dev)
            self.out = torch.zeros((K, 65, 6), dtype=torch.int32, device=dev)
            self.stream = torch.cuda.Stream(device=dev)
            self.host = []
            self.wall = []

        def run(self, n):
            torch.cuda.set_device(dev)
            with torch.cuda.stream(self.stream):
                for _ in range(n):
                    t0 = time.perf_counter()
                    _lib.check(L.aa_sn_run_batch(det._h, _lib.dptr(pcm), offs, lens, K, _lib.dptr(self.ws),
                                                 self.ws.numel(), _lib.dptr(self.out[0, 1:]), 64, 65,
                                                 _lib.dptr(self.out[0, 0]), 65 * 6, _lib.stream_ptr()),
                               "aa_sn_run_batch")
                    t1 = time.perf_counter()
                    self.stream.synchronize()
                    t2 = time.perf_counter()
                    self.host.append(t1 - t0)
                    self.wall.append(t2 - t0)

    one = Lane()
    one.run(2)
    one.host.clear()
    one.wall.clear()
    one.run(reps)
    h = sorted(one.host)[len(one.host) // 2]
    w = sorted(one.wall)[len(one.wall) // 2]
    print(f"1 thread, K={K}: call returns after {1e3 * h:.2f} ms, batch done after {1e3 * w:.2f} ms "
          f"({1e3 * w / K:.3f} ms per recording)", flush=True)
    lanes = [Lane() for _ in range(T)]
    for ln in lanes:
        ln.run(1)
        ln.host.clear()
        ln.wall.clear()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    th = [threading.Thread(target=ln.run, args=(reps,)) for ln in lanes]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    tot = time.perf_counter() - t0
    hs = sorted(x for ln in lanes for x in ln.host)
    print(f"{T} threads, K={K}: call returns after {1e3 * hs[len(hs) // 2]:.2f} ms (median), "
          f"{T * reps * K} recordings in {1e3 * tot:.1f} ms = {1e3 * tot / (T * reps * K):.3f} ms per recording",
          flush=True)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
