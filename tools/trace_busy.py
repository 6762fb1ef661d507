"""GPU busy fraction of a rocprofv3 kernel trace: the union of the kernels'
[start, end) intervals over the wall time they span, in consecutive windows
(the corpus run's timed part shows as the dense windows at the end), and how
much of the busy time has 2+ kernels in flight.

    python tools/trace_busy.py gpurun_out/c4prof [windows]
"""
import csv
import glob
import sys


def main(path, windows=10):
    f = (glob.glob(path.rstrip("/") + "/*kernel_trace.csv") + glob.glob(path.rstrip("/") + "/*/*kernel_trace.csv"))[0]
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(f)))
    t0, t1 = iv[0][0], max(e for _, e in iv)
    step = (t1 - t0) / windows
    print(f"{len(iv)} kernels over {(t1 - t0) / 1e6:.1f} ms")
    for w in range(windows):
        a, b = t0 + w * step, t0 + (w + 1) * step
        ev = []
        for s, e in iv:
            s, e = max(s, a), min(e, b)
            if e > s:
                ev += [(s, 1), (e, -1)]
        ev.sort()
        busy = multi = 0.0
        depth, last = 0, a
        for t, d in ev:
            if depth >= 1:
                busy += t - last
            if depth >= 2:
                multi += t - last
            depth += d
            last = t
        n = sum(1 for s, e in iv if a <= s < b)
        print(f"window {w}: {n:6d} kernels  busy {busy / step:6.1%}  2+ in flight {multi / step:6.1%}")


if __name__ == "__main__":
    main(sys.argv[1], *(int(a) for a in sys.argv[2:]))
