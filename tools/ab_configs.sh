#!/bin/bash
# A/B: each gpu_ab/*.so on the BASELINE config scenes (short runs), PASSES interleaved passes.
set -u
mkdir -p gpurun_out
for pass in $(seq 1 ${PASSES:-2}); do
for cfg in ${AB_CONFIGS:-coffee spaceship lamp}; do
for lib in gpu_ab/*.so; do
  n=$(basename $lib .so)
  DCRT_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps ${AB_STEPS:-6} --warmup 1 --no-cpu-baseline --roofline-images 1 > gpurun_out/abc_${cfg}_$n.log 2>&1 || exit $?
  echo "$cfg $n $(python -c "import json;d=json.load(open('gpurun_out/abc_${cfg}_$n.log'));print(d['ms_per_spp'], d['roofline']['avg_launch_us'])")"
done
done
done
