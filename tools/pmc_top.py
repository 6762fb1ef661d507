"""Per-dispatch rocprofv3 --pmc summary of the last N dispatches of a run
(one step of a many-kernel program), the longest first: counter groups from
several passes (directories) joined on the dispatch's position from the end.
usage: python tools/pmc_top.py N TOP DIR [DIR ...]"""
import collections
import csv
import glob
import sys

n_last, top = int(sys.argv[1]), int(sys.argv[2])
per = []  # per pass: list of (kernel, dur_us, {counter: value}) in dispatch order
for path in sys.argv[3:]:
    files = glob.glob(path.rstrip("/") + "/*counter_collection.csv") + glob.glob(path.rstrip("/") + "/*/*counter_collection.csv")
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            agg[d][r["Counter_Name"]] += float(r["Counter_Value"])
            extra = " ".join(f"{k}={r[k]}" for k in ("Grid_Size", "LDS_Block_Size", "VGPR_Count", "Accum_VGPR_Count", "Scratch_Size") if k in r)
            meta[d] = (r["Kernel_Name"][:70] + "  " + extra, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    ids = sorted(meta)[-n_last:]
    per.append([(meta[d][0], meta[d][1], agg[d]) for d in ids])
rows = []
for i in range(min(len(p) for p in per)):
    k, dur, c = per[0][i]
    merged = dict(c)
    for p in per[1:]:
        if p[i][0] == k:
            merged.update(p[i][2])
    rows.append((dur, k, merged))
for dur, k, c in sorted(rows, key=lambda r: -r[0])[:top]:
    print(f"{k}  dur={dur:.1f}us")
    for name, v in sorted(c.items()):
        print(f"   {name:28s} {v:16.0f}")
