#!/bin/bash
# Shader-core PMC passes (one counter group per pass) over a short bench run.
set -u
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOTDIR/gpurun_out/sq"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "VALUUtilization" "VALUBusy" "SQ_INSTS_VALU SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" "SQ_INSTS_VMEM_RD SQ_INSTS_LDS" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" ${PMC_EXTRA:-}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -f csv -d "$OUT" -o pass$i -- \
      python3 "$ROOTDIR/bench.py" --steps 2 --warmup 1 --roofline-images 1 --no-cpu-baseline > "$OUT/pass$i.log" 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
