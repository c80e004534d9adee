#!/bin/bash
# One PMC pass (PMC_COUNTERS, default VALU instructions / waves / wave cycles / GRBM) per
# experimental library gpu_ab/*.so over a short one-pipeline bench; prints, per library,
# KERNEL's (default material_kernel) n-th non-trivial dispatch (DISPATCH, default 1 = the
# first pass after the camera rays) as counters per wave.
set -u
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
cd /tmp
for lib in "$ROOTDIR"/gpu_ab/*.so; do
  n=$(basename "$lib" .so)
  OUT="$ROOTDIR/gpurun_out/pmcl_$n"
  mkdir -p "$OUT"
  DCRT_LIB=$lib timeout -k 10 120 rocprofv3 --pmc ${PMC_COUNTERS:-SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE} \
      --kernel-trace -f csv -d "$OUT" -o p -- python3 "$ROOTDIR/bench.py" --steps 8 --warmup 0 --streams 1 \
      --roofline-images 1 --no-cpu-baseline > "$OUT/bench.log" 2>&1 || exit $?
  python3 - "$OUT/p_counter_collection.csv" "$n" "${KERNEL:-material_kernel}" "${DISPATCH:-1}" <<'PY'
import collections, csv, sys
per = collections.OrderedDict()
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[3] not in r["Kernel_Name"]:
        continue
    d = per.setdefault(int(r["Dispatch_Id"]), {})
    d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
big = [d for _, d in sorted(per.items()) if d.get("SQ_WAVES", 0) > 1000 and d.get("GRBM_GUI_ACTIVE", 0) > 400000]
d = big[int(sys.argv[4])] if len(big) > int(sys.argv[4]) else {}
w = max(1.0, d.get("SQ_WAVES", 1.0))
print(sys.argv[2], " ".join(f"{k}={v / w:.0f}/wave" for k, v in d.items() if k not in ("SQ_WAVES", "GRBM_GUI_ACTIVE")),
      f"GRBM/xcd={d.get('GRBM_GUI_ACTIVE', 0) / 8:.0f}", f"waves={w:.0f}")
PY
done
