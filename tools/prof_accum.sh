#!/bin/bash
# kernel trace of tools/accum_cost.py (the ordered film pass of interleaved pipelines)
set -e
export TMPDIR=/tmp
ROOTDIR=$(pwd)
mkdir -p gpurun_out/prof_accum
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$ROOTDIR/gpurun_out/prof_accum" -o accum -- python3 "$ROOTDIR/tools/accum_cost.py" > "$ROOTDIR/gpurun_out/prof_accum/log.txt" 2>&1
cd "$ROOTDIR"
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_accum/**/accum_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us avg", round(float(r["TotalDurationNs"]) / 1e6, 2), "ms total")
PY
