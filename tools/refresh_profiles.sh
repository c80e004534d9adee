#!/bin/bash
# GPU box: kernel-trace + PMC profiles of the 20- and 64-image bench workloads (one
# pipeline), their HBM-traffic summaries into profiles/ (so the bench lines below match
# them), then the default and the --steps 20 bench lines. Copy the outputs named in the
# last lines into profiles/rNN_* afterwards.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PMC=1 PROF_STEPS="20 64" bash tools/profile.sh || exit $?
python tools/pmc_traffic.py gpurun_out/prof_20 gpurun_out/${TAG:-r02}_i20 || exit $?
python tools/pmc_traffic.py gpurun_out/prof_64 gpurun_out/${TAG:-r02}_i64 || exit $?
cp gpurun_out/${TAG:-r02}_i20_pmc_traffic.json gpurun_out/${TAG:-r02}_i64_pmc_traffic.json profiles/
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s20.json 2> gpurun_out/bench_s20.err || exit $?
python - <<'PY'
import json
for f in ("gpurun_out/bench_default.json", "gpurun_out/bench_s20.json"):
    d = json.load(open(f)); r = d["roofline"]
    print(f, d["ms_per_spp"], d["value"], r["frac"], r["avg_launch_us"], r["hbm_measured"], r["traffic_source"][:48])
PY
