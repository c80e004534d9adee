#!/bin/bash
# Cast workgroups per CU sweep (DCRT_CAST_BLOCKS_PER_CU = 1..5) on the default bench (GPU box);
# one log per setting under gpurun_out/blk_*.log.
set -u
mkdir -p gpurun_out
for b in 1 2 3 4 5; do
  DCRT_CAST_BLOCKS_PER_CU=$b timeout -k 10 200 python bench.py --steps 24 --warmup 2 --no-cpu-baseline --roofline-images 1 > gpurun_out/blk_$b.log 2>&1 || exit $?
  echo "$b $(python -c "import json;d=json.load(open('gpurun_out/blk_$b.log'));print(d['ms_per_spp'], d['roofline']['avg_launch_us'])")"
done
