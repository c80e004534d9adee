#!/bin/bash
# A/B (round 6): film pass tiles of 16x16 (256 threads) vs 8x8 (64 threads): more independent image
# chains for a band's ordered pass
set -e
DCRT_LIB=gpu_ab/b_tile8.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "film or interleaved or accumulate or bench_configuration or balanced or rank_share or image_batches or filter or frame_loop" > gpurun_out/r06_tile8_parity.txt 2>&1
tail -1 gpurun_out/r06_tile8_parity.txt
for lib in gpu_ab/a_tile16.so gpu_ab/b_tile8.so; do echo "== $lib"; DCRT_LIB=$lib timeout -k 10 200 python tools/accum_cost.py | tail -2; done
AB_STEPS=20 tools/ab_libs.sh
