#!/bin/bash
# Traversal refill/park thresholds (DCRT_TRAVERSAL_TUNE="refill,park") on every BASELINE
# config (tools/bench_configs.py, two pipelines, 16 spp): one JSON line per (tune, config)
# into gpurun_out/tune_configs.jsonl. Each GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/tune_configs.jsonl
: > $OUT
for rep in $(seq 1 ${REPEATS:-1}); do
for t in ${TUNES:-16,32 32,24 36,24}; do
  DCRT_TRAVERSAL_TUNE=$t timeout -k 10 300 python tools/bench_configs.py --spp ${SPP:-16} > gpurun_out/tune_$t.log 2>&1
  rc=$?; echo "tune $t rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "
import json,sys
for l in open('gpurun_out/tune_$t.log'):
    if l.startswith('{'):
        d=json.loads(l); d['tune']='$t'; d['rep']=$rep; print(json.dumps(d))
        print('$t', d['config'], d['ms_per_spp'], d['roofline']['avg_launch_us'], file=sys.stderr)
" >> $OUT
done
done
