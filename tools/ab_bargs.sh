#!/bin/bash
# A/B over bench.py argument variants: each line of $AB_VARIANTS is "name --arg value ...";
# configs in AB_CONFIGS, PASSES interleaved passes. Prints name, config, median ms/spp, repeats.
set -u
mkdir -p gpurun_out
for pass in $(seq 1 ${PASSES:-2}); do
for cfg in ${AB_CONFIGS:-spaceship}; do
while read -r name args; do
  [ -z "$name" ] && continue
  timeout -k 10 200 python bench.py --config $cfg --steps ${AB_STEPS:-16} --warmup 1 --no-cpu-baseline \
      --spaceship-spp 0 --roofline-images 1 $args > gpurun_out/abb_${name}_$cfg.log 2>&1 || exit $?
  echo "$name $cfg $(python -c "import json;d=json.load(open('gpurun_out/abb_${name}_$cfg.log'));print(d['ms_per_spp'], d['repeat_ms_per_spp'])")"
done <<< "${AB_VARIANTS}"
done
done
