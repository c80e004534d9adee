"""Average PMC counters per kernel from tools/pmc_sq.sh output (gpurun_out/sq)."""
import collections
import csv
import glob
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sq"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/pass*_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").replace("dcrt::dev::", "").split("(")[0]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(agg):
    if not any(x in k for x in ("extension", "shadow", "material", "control", "cast")):
        continue
    print(k)
    for c, v in sorted(agg[k].items()):
        print(f"   {c:28s} {sum(v) / len(v):16.1f}")
