#!/bin/bash
# VALU lane utilisation and issue fraction per kernel (one PMC pass per config), one pipeline.
#   lane util = SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64); issue = SQ_INSTS_VALU x 2 / (GRBM_GUI_ACTIVE / 8 x 1024)
set -u
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOTDIR/gpurun_out/lu"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for spec in "cornell 8" "spaceship 4" "spaceship_close 2" "coffee 4"; do
  set -- $spec
  timeout -s KILL 300 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -f csv -d "$OUT" -o "$1" -- \
      python3 "$ROOTDIR/bench.py" --config "$1" --steps "$2" --warmup 0 --no-cpu-baseline --streams 1 --repeats 1 --spaceship-spp 0 --roofline-images 1 > "$OUT/$1.log" 2>&1
  rc=$?; echo "$1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - "$OUT" <<'PY'
import collections, csv, glob, os, sys
d = sys.argv[1]
for f in sorted(glob.glob(f"{d}/*counter_collection.csv")):
    cfg = os.path.basename(f).split("_counter")[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").replace("dcrt::dev::", "").split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k].add(r["Dispatch_Id"])
    for k, c in sorted(agg.items()):
        if not any(x in k for x in ("cast", "material", "control")) or not c.get("SQ_ACTIVE_INST_VALU"):
            continue
        m = len(n[k])
        lu = c["SQ_THREAD_CYCLES_VALU"] / (c["SQ_ACTIVE_INST_VALU"] * 64)
        iss = c["SQ_INSTS_VALU"] * 2 / (c["GRBM_GUI_ACTIVE"] / 8 * 1024)
        print(f"{cfg:16s} {k:48s} lane util {lu:.3f}  valu issue {iss:.3f}  VALU insts/dispatch {c['SQ_INSTS_VALU'] / m:.4g}")
PY
