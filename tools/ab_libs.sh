#!/bin/bash
# A/B: bench each experimental library variant (gpu_ab/*.so) on the GPU box, PASSES
# (default 2) interleaved passes. Prints name, ms/spp, avg cast launch us, avg MATERIAL launch us.
set -u
mkdir -p gpurun_out
for pass in $(seq 1 ${PASSES:-2}); do
for lib in gpu_ab/*.so; do
  n=$(basename $lib .so)
  DCRT_LIB=$lib timeout -k 10 200 python bench.py --steps ${AB_STEPS:-24} --warmup 2 --no-cpu-baseline --roofline-images ${AB_ROOF_IMAGES:-1} --spaceship-spp 0 ${BENCH_ARGS:-} > gpurun_out/ab_$n.log 2>&1 || exit $?
  echo "$n $(python -c "import json;d=json.loads([l for l in open('gpurun_out/ab_$n.log') if l.startswith('{')][-1]);print(d['ms_per_spp'], d['roofline']['avg_launch_us'], d['material']['avg_launch_us'])")"
done
done
