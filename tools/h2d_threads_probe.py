"""Host time of pinned -> device copies issued from several threads at once
(the corpus lanes' upload: 32 per batch, 5.76 MB each, non_blocking, each
lane on its own copy stream), against one thread alone: does the call return
before the DMA runs, and does it stay so under concurrency?

    python tools/h2d_threads_probe.py [threads] [copies] [MB]
"""
import sys
import threading
import time

import torch


def main(T=8, n=32, mb=5.76):
    dev = torch.device("cuda", 0)
    nb = int(mb * 1e6) // 2 * 2
    src = [torch.empty(nb, dtype=torch.uint8, pin_memory=True) for _ in range(n)]
    dst = [torch.empty(nb * n, dtype=torch.uint8, device=dev) for _ in range(T)]
    streams = [torch.cuda.Stream(device=dev) for _ in range(T)]

    def lane(j, out):
        torch.cuda.set_device(dev)
        with torch.cuda.stream(streams[j]):
            t0 = time.perf_counter()
            for i in range(n):
                dst[j][i * nb:(i + 1) * nb].copy_(src[i], non_blocking=True)
            t1 = time.perf_counter()
            streams[j].synchronize()
            t2 = time.perf_counter()
        out[j] = (t1 - t0, t2 - t0)

    for threads in (1, T):
        for rep in range(3):
            out = [None] * threads
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            th = [threading.Thread(target=lane, args=(j, out)) for j in range(threads)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            wall = time.perf_counter() - t0
            issue = max(o[0] for o in out)
            gb = threads * n * nb / 1e9
            print(f"threads={threads} rep={rep}: {n} copies of {nb / 1e6:.2f} MB per thread; calls return after "
                  f"{1e3 * issue:.2f} ms (max over threads, {1e3 * issue / n:.3f} ms per call); all done after "
                  f"{1e3 * wall:.2f} ms = {gb / wall:.1f} GB/s", flush=True)


if __name__ == "__main__":
    main(*(float(a) if "." in a else int(a) for a in sys.argv[1:]))
