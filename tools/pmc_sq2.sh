#!/bin/bash
# Latency / stall PMC passes on a short bench run (one group per pass).
set -u
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOTDIR/gpurun_out/sq2"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQ_WAIT_ANY SQ_WAVE_CYCLES" "SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY" "TCP_TOTAL_ACCESSES_sum TCP_TCC_READ_REQ_sum" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCP_LATENCY_sum TCP_TCC_READ_REQ_LATENCY_sum" "SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -f csv -d "$OUT" -o pass$i -- \
      python3 "$ROOTDIR/bench.py" --steps 2 --warmup 1 --roofline-images 1 --no-cpu-baseline > "$OUT/pass$i.log" 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
