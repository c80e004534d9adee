#!/bin/bash
# PMC passes over a short one-pipeline bench run, one pass per counter group. Groups are
# separated by ';' in PMC_GROUPS (each within the per-block slot limits:
# 8 SQ, 4 TCC, 4 TCP, 2 GRBM). Output: gpurun_out/${PMC_OUT:-pmcg}/passN_*.
# Summarise one kernel's median dispatch with tools/sq_dispatch.py gpurun_out/pmcg <name>.
set -u
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOTDIR/gpurun_out/${PMC_OUT:-pmcg}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
IFS=';' read -ra groups <<< "${PMC_GROUPS:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE}"
for grp in "${groups[@]}"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace -f csv -d "$OUT" -o pass$i -- \
      python3 "$ROOTDIR/bench.py" --steps ${PMC_IMAGES:-8} --warmup 0 --streams 1 --roofline-images 1 --no-cpu-baseline \
      ${BENCH_ARGS:-} > "$OUT/pass$i.log" 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
