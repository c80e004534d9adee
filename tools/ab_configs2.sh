#!/bin/bash
# A/B over configs: bench.py for each gpu_ab/*.so on each config in AB_CONFIGS (default
# "spaceship cornell"), PASSES interleaved passes. Prints lib, config, ms/spp, cast launch us.
set -u
mkdir -p gpurun_out
for pass in $(seq 1 ${PASSES:-2}); do
for cfg in ${AB_CONFIGS:-spaceship cornell}; do
for lib in gpu_ab/*.so; do
  n=$(basename $lib .so)
  steps=${AB_STEPS:-16}
  DCRT_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps $steps --warmup 1 --no-cpu-baseline \
      --spaceship-spp 0 --roofline-images 2 ${BENCH_ARGS:-} > gpurun_out/ab_${n}_$cfg.log 2>&1 || exit $?
  echo "$n $cfg $(python -c "import json;d=json.load(open('gpurun_out/ab_${n}_$cfg.log'));print(d['ms_per_spp'], d['repeat_ms_per_spp'], d['roofline']['avg_launch_us'])")"
done
done
done
