#!/bin/bash
# A/B over library variants (gpu_ab/*.so) x environment variants ($AB_VARIANTS lines "name ENV=value ...")
# on the configs in AB_CONFIGS, PASSES interleaved passes. Prints lib, env, config, ms/spp, repeats.
set -u
mkdir -p gpurun_out
for pass in $(seq 1 ${PASSES:-1}); do
for cfg in ${AB_CONFIGS:-cornell}; do
for lib in gpu_ab/*.so; do
n=$(basename $lib .so)
while read -r name envs; do
  [ -z "$name" ] && continue
  env DCRT_LIB=$lib $envs timeout -k 10 200 python bench.py --config $cfg --steps ${AB_STEPS:-16} --warmup 1 --no-cpu-baseline \
      --spaceship-spp 0 --roofline-images 1 ${BENCH_ARGS:-} > gpurun_out/able_${n}_${name}_$cfg.log 2>&1 || exit $?
  echo "$n $name $cfg $(python -c "import json;d=json.load(open('gpurun_out/able_${n}_${name}_$cfg.log'));print(d['ms_per_spp'], d['repeat_ms_per_spp'], d['roofline']['avg_launch_us'])")"
done <<< "${AB_VARIANTS}"
done
done
done
