#!/bin/bash
# A/B: bench the in-tree library under environment variants. Each line of $AB_VARIANTS
# is "name ENV=value ..." (name alone = defaults).
set -u
mkdir -p gpurun_out
while read -r name envs; do
  [ -z "$name" ] && continue
  env $envs timeout -k 10 200 python bench.py --steps 24 --warmup 2 --no-cpu-baseline --roofline-images 1 ${BENCH_ARGS:-} > gpurun_out/abenv_$name.log 2>&1 || exit $?
  echo "$name $(python -c "import json;d=json.load(open('gpurun_out/abenv_$name.log'));print(d['ms_per_spp'], d['roofline']['avg_launch_us'], d['roofline']['frac'])")"
done <<< "${AB_VARIANTS}"
