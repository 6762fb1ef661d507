"""Print a rocprofv3 --stats kernel summary (CSV) as a table."""
import csv
import glob
import sys

path = sys.argv[1]
files = glob.glob(path) if ("*" in path or not path.endswith(".csv")) else [path]
files = [f for f in files if f.endswith(".csv")]
if not files:
    files = glob.glob(path.rstrip("/") + "/*_kernel_stats.csv") + glob.glob(path.rstrip("/") + "/*/*_kernel_stats.csv")
for f in files:
    rows = list(csv.DictReader(open(f)))
    print(f"{'kernel':64s} {'calls':>6s} {'avg_us':>9s} {'min_us':>9s} {'tot%':>6s}")
    for x in rows:
        print(f"{x['Name'][:64]:64s} {x['Calls']:>6s} {float(x['AverageNs'])/1e3:9.2f} "
              f"{float(x['MinNs'])/1e3:9.2f} {float(x['Percentage']):6.2f}")
