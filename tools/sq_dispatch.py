"""Per-dispatch PMC values for one kernel from tools/pmc_sq.sh output: the counters of the
slowest and the median dispatch (e.g. CONTROL with and without NEW_PATH work)."""
import collections
import csv
import glob
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sq"
name = sys.argv[2] if len(sys.argv) > 2 else "control_kernel"
per = collections.defaultdict(dict)        # (pass, dispatch) -> counter -> value
for f in glob.glob(f"{d}/pass*_counter_collection.csv"):
    p = f.split("/")[-1].split("_")[0]
    for r in csv.DictReader(open(f)):
        if name not in r["Kernel_Name"]:
            continue
        per[(p, int(r["Dispatch_Id"]))][r["Counter_Name"]] = per[(p, int(r["Dispatch_Id"]))].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
bypass = collections.defaultdict(list)
for (p, _), cs in sorted(per.items()):
    bypass[p].append(cs)
for p, lst in sorted(bypass.items()):
    key = next(iter(lst[0]))
    lst.sort(key=lambda cs: cs[key])
    hi, med = lst[-1], lst[len(lst) // 2]
    for c in sorted(hi):
        print(f"{p:7s} {c:28s} max {hi[c]:16.1f}   median {med[c]:16.1f}")
