#!/bin/bash
# Traversal refill / park threshold sweep on the default Cornell bench (GPU box):
# DCRT_TRAVERSAL_TUNE="refill,park" per run; prints ms/spp and the cast launch time per setting.
#   TUNES="32,24 36,24" bash tools/sweep_tune.sh
set -u
mkdir -p gpurun_out
for t in ${TUNES:-16,32 24,32 32,32 40,32 48,32 32,24 32,40 32,48}; do
  DCRT_TRAVERSAL_TUNE=$t timeout -k 10 200 python bench.py --steps 24 --warmup 2 --no-cpu-baseline --roofline-images 1 > gpurun_out/sweep_$t.log 2>&1 || exit $?
  echo "$t $(python -c "import json;d=json.load(open('gpurun_out/sweep_$t.log'));print(d['ms_per_spp'], d['roofline']['avg_launch_us'])")"
done
