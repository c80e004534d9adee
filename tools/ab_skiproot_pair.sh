#!/bin/bash
# A/B (round 6): the root's sure hit for the pair traversal (trav_skip_root_pair), spaceship configs
set -e
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_random_scenes.py -k "spaceship or pair or config" > gpurun_out/r06_skippair_parity.txt 2>&1
tail -1 gpurun_out/r06_skippair_parity.txt
export AB_CONFIGS="spaceship_close spaceship" AB_STEPS=8 PASSES=2
export AB_VARIANTS="skip
noskip DCRT_SKIP_ROOT=0"
tools/ab_env2.sh
