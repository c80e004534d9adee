#!/bin/bash
# ADVICE r05 follow-up: visits per phase-A check (2 / 3 / 4) with the ring's corrected bounds:
# ring / spaceship parity on the 4-visit library, then an interleaved A/B on Cornell and the close framing
set -e
DCRT_LIB=gpu_ab/b_vpc4.so timeout -k 10 400 python -u -m pytest -q -rf --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "ring or spaceship or traversal_counters" > gpurun_out/r06_vpc4_parity.txt 2>&1 || true
grep -E "^FAILED|passed|failed" gpurun_out/r06_vpc4_parity.txt || true
AB_STEPS=20 tools/ab_libs.sh
BENCH_ARGS="--config spaceship_close" AB_STEPS=8 tools/ab_libs.sh
