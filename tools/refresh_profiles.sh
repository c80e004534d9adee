#!/bin/bash
# GPU box: kernel-trace + PMC profiles (tools/prof_config.sh, one pipeline) of the three
# workloads the bench's roofline objects are quoted on -- Cornell 1080p 20 and 64 images
# (the driver's --steps 20 and the default) and the spaceship leg (4K, 16 images) -- their
# HBM-traffic summaries into profiles/${TAG}_*_pmc_traffic.json (bench.py matches its runs
# against them), then the default and the --steps 20 bench lines. The new profiles are
# also copied under gpurun_out/profiles/ (what gpurun brings back) for committing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03}
mkdir -p gpurun_out profiles
for w in "cornell 20 c20" "cornell 64 c64" "spaceship 16 s16"; do
  set -- $w
  CONFIG=$1 STEPS=$2 OUT=gpurun_out/prof_$3 tools/prof_config.sh || exit $?
  python tools/pmc_traffic.py gpurun_out/prof_$3 profiles/${TAG}_$3 || exit $?
  cp gpurun_out/prof_$3/trace_kernel_stats.csv profiles/${TAG}_$3_kernel_stats.csv
  mkdir -p gpurun_out/profiles
  cp profiles/${TAG}_$3_kernel_stats.csv profiles/${TAG}_$3_pmc_traffic.json gpurun_out/profiles/
done
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s20.json 2> gpurun_out/bench_s20.err || exit $?
python - <<'PY'
import json
for f in ("gpurun_out/bench_default.json", "gpurun_out/bench_s20.json"):
    d = json.load(open(f)); r = d["roofline"]; s = d.get("spaceship", {}).get("roofline", {})
    print(f, d["ms_per_spp"], d["value"], r["frac"], r["avg_launch_us"], r["traffic_source"][:40], s.get("frac"), s.get("traffic_source", "")[:40])
PY
