#!/bin/bash
# Round-end measurements (GPU box): the driver's --steps 20 line, the default line, and every
# BASELINE config at 16 spp (one JSON line each), each under its own time limit.
set -e
TAG=${TAG:-r06}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 > gpurun_out/${TAG}_bench_s20.json
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench_default.json
: > gpurun_out/${TAG}_configs.jsonl
for c in cornell coffee "coffee --no-multiscattering" spaceship spaceship_close lamp; do
  timeout -k 10 300 python bench.py --config $c --steps 16 --no-cpu-baseline --spaceship-spp 0 >> gpurun_out/${TAG}_configs.jsonl
done
