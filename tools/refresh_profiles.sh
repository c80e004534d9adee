#!/bin/bash
# GPU box: kernel-trace + PMC profiles (tools/prof_config.sh, one pipeline) of the workloads the
# bench's roofline / material / pipeline objects are quoted on, their HBM-traffic summaries into
# profiles/${TAG}_<key>_pmc_traffic.json (bench.py matches its runs against them) and the kernel
# stats beside them. WORKLOADS = "config steps key [extra bench args]" entries separated by ';'
# (default: Cornell 20 and 64 images -- the driver's --steps 20 and the default -- and the
# spaceship leg, 4K 16 images). Copies land under gpurun_out/profiles/ (what gpurun brings back).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04}
mkdir -p gpurun_out/profiles profiles
# (prof_config runs one pipeline: --pool gives it the bench's whole pool -- three Cornell
# pipelines of 2^24, two coffee ones -- so the recorded workload key is the bench's)
IFS=';' read -ra ITEMS <<< "${WORKLOADS:-cornell 20 c20 --pool 50331648;cornell 64 c64 --pool 50331648;spaceship 16 s16}"
for w in "${ITEMS[@]}"; do
  set -- $w
  cfg=$1 steps=$2 key=$3; shift 3
  PROF_ARGS="$*" CONFIG=$cfg STEPS=$steps OUT=gpurun_out/prof_$key tools/prof_config.sh || exit $?
  python tools/pmc_traffic.py gpurun_out/prof_$key profiles/${TAG}_$key || exit $?
  cp gpurun_out/prof_$key/trace_kernel_stats.csv profiles/${TAG}_${key}_kernel_stats.csv
  cp profiles/${TAG}_${key}_kernel_stats.csv profiles/${TAG}_${key}_pmc_traffic.json gpurun_out/profiles/
done
