#!/bin/bash
# Round 6 A/B: the film pass software-pipelined over a batch's images (double-buffered LDS tile,
# next image's loads in flight, s_barrier without the fence's vmcnt wait)
set -e
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "film or interleaved or accumulate or bench_configuration or balanced or rank_share or image_batches or filter" > gpurun_out/r06_film2_parity.txt 2>&1
tail -1 gpurun_out/r06_film2_parity.txt
for lib in gpu_ab/a_base.so gpu_ab/b_film2.so; do echo "== $lib"; DCRT_LIB=$lib timeout -k 10 200 python tools/accum_cost.py | tail -2; done
AB_STEPS=20 tools/ab_libs.sh
