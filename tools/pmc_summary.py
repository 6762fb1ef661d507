"""Summarise rocprofv3 --pmc counter_collection.csv: last dispatch per kernel."""
import collections
import csv
import glob
import sys

for path in sys.argv[1:]:
    for f in glob.glob(path.rstrip("/") + "/*counter_collection.csv") + glob.glob(path.rstrip("/") + "/*/*counter_collection.csv"):
        rows = list(csv.DictReader(open(f)))
        agg = collections.defaultdict(float)
        meta = {}
        for r in rows:
            agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            meta[r["Dispatch_Id"]] = (r["Kernel_Name"][:110], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        last = {}
        for d, (k, _) in meta.items():
            if k not in last or int(d) > int(last[k]):
                last[k] = d
        for k, d in last.items():
            print(f"{k}  dur={meta[d][1]/1e3:.1f}us")
            for (dd, c), v in sorted(agg.items()):
                if dd == d:
                    print(f"   {c:28s} {v:16.0f}")
