#!/bin/bash
# A/B over configs and environment variants of the in-tree library: each line of
# $AB_VARIANTS is "name ENV=value ..." (name alone = defaults); configs in AB_CONFIGS.
# Prints name, config, median ms/spp and the repeats.
set -u
mkdir -p gpurun_out
for pass in $(seq 1 ${PASSES:-2}); do
for cfg in ${AB_CONFIGS:-cornell spaceship coffee}; do
while read -r name envs; do
  [ -z "$name" ] && continue
  env $envs timeout -k 10 200 python bench.py --config $cfg --steps ${AB_STEPS:-16} --warmup 1 --no-cpu-baseline \
      --spaceship-spp 0 --roofline-images 1 ${BENCH_ARGS:-} > gpurun_out/abenv_${name}_$cfg.log 2>&1 || exit $?
  echo "$name $cfg $(python -c "import json;d=json.load(open('gpurun_out/abenv_${name}_$cfg.log'));print(d['ms_per_spp'], d['repeat_ms_per_spp'])")"
done <<< "${AB_VARIANTS}"
done
done
