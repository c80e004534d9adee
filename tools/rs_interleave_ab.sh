#!/bin/bash
# rank_sim (round 6): image-interleaved pipelines over one cost-balanced band per rank, without
# and with a calibration round; every rank resident, repeats round-robin, median of 5 per rank
set -e
R="python tools/rank_sim.py --steps 20 --repeats 5 --streams 3 --pool 50331648"
echo "== bands N1"; timeout -k 10 150 $R --gpus 1
echo "== inter B1 calib0"; timeout -k 10 300 $R --gpus 2,4,8 --interleave --bands-per-rank 1
echo "== inter B1 calib1"; timeout -k 10 400 $R --gpus 2,4,8 --interleave --bands-per-rank 1 --calibrate 1
