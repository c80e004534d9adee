set -e
R="python tools/rank_sim.py --steps 20"
for v in base nb; do
  if [ $v = nb ]; then export DCRT_BATCH_POOL_LIMIT=0 DCRT_MAX_BATCH=256; else unset DCRT_BATCH_POOL_LIMIT DCRT_MAX_BATCH; fi
  echo "== $v N1 s3"; timeout -k 10 120 $R --gpus 1 --streams 3 --pool 50331648
  echo "== $v N8 s2"; timeout -k 10 200 $R --gpus 8 --streams 2 --pool 33554432
  echo "== $v N8 s3"; timeout -k 10 200 $R --gpus 8 --streams 3 --pool 50331648
done
