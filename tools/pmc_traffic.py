"""Per-launch HBM bytes of one bench step from rocprofv3 --pmc runs.

usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json

FETCH_DIR / WRITE_DIR hold the counter_collection.csv of
`rocprofv3 --pmc FETCH_SIZE` and `rocprofv3 --pmc WRITE_SIZE` runs of
`bench.py` (separate passes: FETCH_SIZE takes 3 of the 4 TCC slots).  The
counters are in KiB.  Per MI355X_MICROARCH.md (HBM section) FETCH_SIZE on
gfx950 reports half the bytes of a coalesced streaming read, so it is doubled;
WRITE_SIZE is taken as is.  (Calibration in this workload: fe_stats streams
every PCM sample of the step once with float4 loads, and 2 x FETCH_SIZE equals
the 19.0 MB of distinct PCM its 64 windows cover.)

The output lists the kernels of the LAST complete step (fe_stats ... track_mean)
in dispatch order, which is how bench.py maps them onto its launches.
"""
import collections
import csv
import glob
import json
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__) + "/..")


def dispatches(d):
    files = glob.glob(d.rstrip("/") + "/*counter_collection.csv") + \
        glob.glob(d.rstrip("/") + "/*/*counter_collection.csv")
    vals = collections.defaultdict(float)
    meta = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            i = int(r["Dispatch_Id"])
            vals[i] += float(r["Counter_Value"])
            meta[i] = (r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return [(i, meta[i][0], vals[i], meta[i][1]) for i in sorted(meta)]


def last_step(ds):
    starts = [k for k, d in enumerate(ds) if "fe_stats" in d[1]]
    if len(starts) < 2:
        raise SystemExit("need at least two steps in the profile")
    # the last fe_stats whose step runs through to track_mean; runtime copies
    # (__amd_rocclr_copyBuffer: parity read-backs, clip-pair rotation) that
    # land inside the window are not launches of the step and are dropped
    for a in reversed(starts):
        step = []
        for d in ds[a:]:
            if "aa::" not in d[1]:
                continue
            if "fe_stats" in d[1] and step:
                break
            step.append(d)
            if "track_mean" in d[1]:
                return step
    raise SystemExit("no complete step (fe_stats ... track_mean) in the profile")


def main():
    fetch, write, out = sys.argv[1:4]
    precision = sys.argv[4] if len(sys.argv) > 4 else "bf16"
    f = last_step(dispatches(fetch))
    w = last_step(dispatches(write))
    assert [x[1] for x in f] == [x[1] for x in w], "the two passes ran different kernels"
    from bench import WORKLOAD
    kernels = []
    for (_, name, fk, dur), (_, _, wk, _) in zip(f, w):
        fb = 2.0 * fk * 1024.0
        wb = wk * 1024.0
        if "head_final" in name and kernels:  # second launch of the head stage: one entry per stage
            k = kernels[-1]
            k["fetch_bytes"] += round(fb)
            k["write_bytes"] += round(wb)
            k["hbm_bytes"] += round(fb + wb)
            k["dur_us_profiled"] = round(k["dur_us_profiled"] + dur, 2)
            continue
        kernels.append({"name": name[:120], "fetch_bytes": round(fb), "write_bytes": round(wb),
                        "hbm_bytes": round(fb + wb), "dur_us_profiled": round(dur, 2)})
    json.dump({"workload": WORKLOAD, "precision": precision,
               "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, "
               f"bench.py --precision {precision} --steps 3 --warmup 2; FETCH_SIZE x2 (gfx950 correction), KiB x 1024",
               "kernels": kernels}, open(out, "w"), indent=1)
    for k in kernels:
        print(f"{k['name'][:60]:60s} fetch {k['fetch_bytes']/1e6:8.2f} MB  write {k['write_bytes']/1e6:8.2f} MB")


if __name__ == "__main__":
    main()
