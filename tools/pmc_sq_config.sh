#!/bin/bash
# Shader-core PMC passes (one counter group per pass) over one bench.py workload:
#   CONFIG=spaceship STEPS=4 OUT=gpurun_out/sq_spaceship tools/pmc_sq_config.sh
# Summarise with: python tools/sq_summary.py gpurun_out/sq_spaceship
set -u
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
CONFIG="${CONFIG:-spaceship}"
STEPS="${STEPS:-4}"
OUT="$ROOTDIR/${OUT:-gpurun_out/sq_$CONFIG}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ARGS="--config $CONFIG --steps $STEPS --warmup 0 --no-cpu-baseline --streams 1 --repeats 1 --spaceship-spp 0 --roofline-images 1 ${PROF_ARGS:-}"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" ${PMC_EXTRA:-}; do
  i=$((i+1))
  grp=${grp//+/ }   # (PMC_EXTRA groups join their counters with +)
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -f csv -d "$OUT" -o pass$i -- \
      python3 "$ROOTDIR/bench.py" $ARGS > "$OUT/pass$i.log" 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
