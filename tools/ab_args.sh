#!/bin/bash
# A/B of bench.py arguments on one box (two passes).
set -u
mkdir -p gpurun_out
i=0
for pass in $(seq 1 ${PASSES:-2}); do
while IFS= read -r args; do
  i=$((i+1))
  timeout -k 10 200 python bench.py --steps 32 --warmup 2 --no-cpu-baseline --roofline-images 1 $args > gpurun_out/abargs_$i.log 2>&1 || exit $?
  echo "$args | $(python -c "import json;d=json.load(open('gpurun_out/abargs_$i.log'));print(d['ms_per_spp'])")"
done <<< "${AB_ARGS:---streams 2
--pool 33554432
--pool 67108864
--iterations 8}"
done
