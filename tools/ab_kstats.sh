#!/bin/bash
# Per-kernel A/B (GPU box): a kernel-trace pass of the one-pipeline S-image bench
# (S = AB_IMAGES, default 64) for each gpu_ab/*.so, PASSES (default 1) interleaved
# passes; prints each library's average duration of the path-tracing kernels in us.
set -u
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
cd /tmp
for pass in $(seq 1 ${PASSES:-1}); do
for lib in "$ROOTDIR"/gpu_ab/*.so; do
  n=$(basename "$lib" .so)
  OUT="$ROOTDIR/gpurun_out/abk_${n}_$pass"
  mkdir -p "$OUT"
  DCRT_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o trace -- \
      python3 "$ROOTDIR/bench.py" --steps ${AB_IMAGES:-64} --warmup 0 --no-cpu-baseline --streams 1 \
      ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1 || exit $?
  python3 - "$OUT/trace_kernel_stats.csv" "$n" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for r in rows:
    name = r["Name"]
    if "lut_integrate" in name or "build_" in name:
        continue
    short = name.split("(")[0].replace("void ", "").replace("dcrt::dev::", "")
    out.append((float(r["TotalDurationNs"]), short, float(r["AverageNs"]) / 1e3, int(r["Calls"])))
out.sort(reverse=True)
print(sys.argv[2], " ".join(f"{s}={a:.1f}us/{c}" for _, s, a, c in out[:5]),
      f"total={sum(t for t, *_ in out) / 1e6:.1f}ms")
PY
done
done
