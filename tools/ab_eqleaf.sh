#!/bin/bash
# A/B (round 6): entry-free order with the equal-box leaf shortcut (descend parks at a near leaf whose
# box is its parent's) against without (DCRT_FLAT_EQ_LEAF=0); Cornell --steps 20
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_random_scenes.py -k "cornell or identity or random or knobs or bench_configuration or traversal_variants or render" > gpurun_out/r06_eqleaf_parity.txt 2>&1
tail -1 gpurun_out/r06_eqleaf_parity.txt
export AB_CONFIGS="cornell" AB_STEPS=20 PASSES=3
export AB_VARIANTS="eq
noeq DCRT_FLAT_EQ_LEAF=0"
tools/ab_env2.sh
