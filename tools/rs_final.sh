#!/bin/bash
# rank_sim record (round 6, final tree): N = 1 (three banded pipelines) and N = 2 / 4 / 8 with the
# bench's N > 1 construction (one calibrated band per rank, three image-interleaved pipelines)
set -e
R="python tools/rank_sim.py --steps 20 --repeats 5 --streams 3 --pool 50331648"
echo "== bands N1"; timeout -k 10 150 $R --gpus 1
echo "== inter B1 calib1"; timeout -k 10 500 $R --gpus 2,4,8 --interleave --bands-per-rank 1 --calibrate 1
echo "== bands N1 again"; timeout -k 10 150 $R --gpus 1
