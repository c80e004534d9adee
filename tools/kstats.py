"""Print a compact per-kernel table from a rocprofv3 *_kernel_stats.csv."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows:
    name = r["Name"].replace("void ", "").replace("dcrt::dev::", "").split("(")[0]
    print(f"{name:40s} calls {int(r['Calls']):6d}  avg {float(r['AverageNs'])/1e3:9.1f} us  "
          f"total {float(r['TotalDurationNs'])/1e6:9.2f} ms  {100*float(r['TotalDurationNs'])/tot:5.1f} %")
