"""Overlay of the corpus lanes' host phases (AA_BATCH_TRACE json, CLOCK_MONOTONIC
ns) on the GPU's busy time (rocprofv3 kernel trace): per window of the timed
run, the GPU busy fraction and how many lanes are in each phase.

    python tools/corpus_timeline.py gpurun_out/c4prof gpurun_out/batch_trace.json [windows]
"""
import collections
import csv
import glob
import json
import sys


def _intervals(trace_dir, kind):
    fs = glob.glob(trace_dir.rstrip("/") + f"/*{kind}_trace.csv") + glob.glob(trace_dir.rstrip("/") + f"/*/*{kind}_trace.csv")
    if not fs:
        return []
    return sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(fs[0])))


def _busy(iv, a, b):
    pts = []
    for s, e in iv:
        s, e = max(s, a), min(e, b)
        if e > s:
            pts += [(s, 1), (e, -1)]
    pts.sort()
    busy, depth, last = 0.0, 0, a
    for t, d in pts:
        if depth >= 1:
            busy += t - last
        depth += d
        last = t
    return busy


def main(trace_dir, events_path, windows=30):
    iv = _intervals(trace_dir, "kernel")
    cp = _intervals(trace_dir, "memory_copy")
    ev = json.load(open(events_path))
    t0 = min(e[2] for e in ev)
    t1 = max(e[3] for e in ev)
    print(f"host phases span {(t1 - t0) / 1e6:.1f} ms; kernels in it: {sum(1 for s, e in iv if t0 <= s < t1)}; "
          f"kernel trace spans [{(iv[0][0] - t0) / 1e6:.1f}, {(max(e for _, e in iv) - t0) / 1e6:.1f}] ms of it")
    step = (t1 - t0) / windows
    names = sorted({e[1] for e in ev})
    print("window   busy  copies " + " ".join(f"{n[:8]:>8s}" for n in names) + "   (lane-ms of each phase in the window)")
    tot_busy = 0.0
    for w in range(windows):
        a, b = t0 + w * step, t0 + (w + 1) * step
        busy = _busy(iv, a, b)
        cbusy = _busy(cp, a, b)
        tot_busy += busy
        ph = collections.Counter()
        for _, n, s, e in ev:
            s, e = max(s, a), min(e, b)
            if e > s:
                ph[n] += (e - s) / 1e6
        print(f"{w:4d}  {busy / step:6.1%} {cbusy / step:6.1%} " + " ".join(f"{ph[n]:8.1f}" for n in names))
    print(f"GPU busy over the host-phase span: {tot_busy / (t1 - t0):.1%}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *(int(a) for a in sys.argv[3:]))
