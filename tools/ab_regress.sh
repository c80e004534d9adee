#!/bin/bash
# same-box A/B of commit libraries (gpu_ab/*.so), Cornell --steps 20 then coffee --steps 16
set -e
PASSES=2 AB_STEPS=20 tools/ab_libs.sh
PASSES=1 AB_STEPS=16 BENCH_ARGS="--config coffee" tools/ab_libs.sh
