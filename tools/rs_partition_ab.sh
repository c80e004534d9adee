#!/bin/bash
# rank_sim of the film partition (round 6): cost-balanced bands vs stripes, median of 3 repeats per rank
set -e
R="python tools/rank_sim.py --steps 20 --repeats 3"
echo "== stripes N1 s3"; timeout -k 10 150 $R --gpus 1 --streams 3 --pool 50331648 --partition stripes
echo "== balanced N1 s3"; timeout -k 10 150 $R --gpus 1 --streams 3 --pool 50331648 --partition balanced
echo "== balanced N2,4,8 s3"; timeout -k 10 400 $R --gpus 2,4,8 --streams 3 --pool 50331648 --partition balanced
echo "== balanced N8 s2"; timeout -k 10 250 $R --gpus 8 --streams 2 --pool 33554432 --partition balanced
echo "== stripes N8 s2"; timeout -k 10 250 $R --gpus 8 --streams 2 --pool 33554432 --partition stripes
