#!/bin/bash
# random-scene parity soak on the final tree (GPU cases only), default kernels, then with the
# entry-free order's empty-node path forced (DCRT_FLAT_MERGE=0)
set -e
DCRT_RANDOM_SCENE_SEEDS=${SEEDS:-100} timeout -k 10 500 python -u -m pytest tests/test_random_scenes.py -m gpu -q --timeout 300 --timeout-method thread -x 2>&1 | tail -2
DCRT_FLAT_MERGE=0 DCRT_RANDOM_SCENE_SEEDS=${SEEDS:-100} timeout -k 10 500 python -u -m pytest tests/test_random_scenes.py -m gpu -q --timeout 300 --timeout-method thread -x -k "lds or obj" 2>&1 | tail -2
