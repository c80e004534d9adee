#!/bin/bash
# rocprofv3 passes over one bench.py workload (GPU box): a kernel trace + stats pass, then
# one pass per PMC group (never combined with other traces). One pipeline (--streams 1),
# no warmup, so every cast launch is one of the roofline leg's workload.
#   CONFIG=spaceship STEPS=8 OUT=gpurun_out/prof_spaceship tools/prof_config.sh
# Summarise with: python tools/pmc_traffic.py $OUT profiles/r03_spaceship
set -u
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
cd /tmp
CONFIG="${CONFIG:-spaceship}"
STEPS="${STEPS:-8}"
OUT="$ROOTDIR/${OUT:-gpurun_out/prof_$CONFIG}"
mkdir -p "$OUT"
ARGS="--config $CONFIG --steps $STEPS --warmup 0 --no-cpu-baseline --streams 1 --repeats 1 --spaceship-spp 0 ${PROF_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o trace -- \
    python3 "$ROOTDIR/bench.py" $ARGS > "$OUT/trace_bench.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
[ -n "${NO_PMC:-}" ] && exit 0
# FETCH_SIZE (3 TCC), WRITE_SIZE (2 TCC), TCC_EA0_RDREQ_sum, L2 hit / miss: separate passes
# (the SQ + GRBM pass: VALU issue per cast launch for the bench's compute statement)
for ctr in FETCH_SIZE WRITE_SIZE TCC_EA0_RDREQ_sum "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE" ${EXTRA_PMC:-}; do
  tag=$(echo "$ctr" | tr ' ' '+')
  timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace -f csv -d "$OUT" -o "pmc_$tag" -- \
      python3 "$ROOTDIR/bench.py" $ARGS > "$OUT/pmc_${tag}.log" 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
