#!/bin/bash
# rank_sim A/B of the film partition (round 6): stripes vs cost-balanced bands, 2 / 3 pipelines per rank
set -e
R="python tools/rank_sim.py --steps 20"
for rep in 1 2; do
echo "== stripes N1 s3"; timeout -k 10 120 $R --gpus 1 --streams 3 --pool 50331648 --partition stripes
echo "== balanced N1 s3"; timeout -k 10 120 $R --gpus 1 --streams 3 --pool 50331648 --partition balanced
echo "== stripes N8 s2"; timeout -k 10 200 $R --gpus 8 --streams 2 --pool 33554432 --partition stripes
echo "== balanced N8 s2"; timeout -k 10 200 $R --gpus 8 --streams 2 --pool 33554432 --partition balanced
echo "== balanced N8 s3"; timeout -k 10 200 $R --gpus 8 --streams 3 --pool 50331648 --partition balanced
done
echo "== balanced N2 s3"; timeout -k 10 200 $R --gpus 2 --streams 3 --pool 50331648 --partition balanced
echo "== balanced N4 s3"; timeout -k 10 200 $R --gpus 4 --streams 3 --pool 50331648 --partition balanced
