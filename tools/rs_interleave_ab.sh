#!/bin/bash
# rank_sim (round 6): image-interleaved pipelines with time-calibrated bands, median of 3 repeats per rank
set -e
R="python tools/rank_sim.py --steps 20 --repeats 3 --streams 3 --pool 50331648"
echo "== bands N1"; timeout -k 10 150 $R --gpus 1
echo "== inter B1 N8 calib8"; timeout -k 10 400 $R --gpus 8 --interleave --bands-per-rank 1 --calibrate 8
echo "== inter B2 N8 calib8"; timeout -k 10 400 $R --gpus 8 --interleave --bands-per-rank 2 --calibrate 8
echo "== inter B1 N2,4 calib8"; timeout -k 10 400 $R --gpus 2,4 --interleave --bands-per-rank 1 --calibrate 8
echo "== bands N8 calib8"; timeout -k 10 400 $R --gpus 8 --calibrate 8
