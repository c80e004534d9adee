#!/bin/bash
# rocprofv3 passes over short bench runs (GPU box). Per image count S in PROF_STEPS
# (default "20 64": the driver's --steps 20 line and the default 64-spp line): a kernel
# trace + stats pass, then (PMC=1) one PMC counter per pass, counters never combined
# with other traces. Outputs under gpurun_out/prof_S; summarise each with
#   python tools/pmc_traffic.py gpurun_out/prof_S profiles/rNN_iS
# The default command (two concurrent pipelines) is traced once into gpurun_out/prof.
set -u
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
cd /tmp
for S in ${PROF_STEPS:-20 64}; do
  OUT="$ROOTDIR/gpurun_out/prof_$S"
  mkdir -p "$OUT"
  # ONE pipeline (--streams 1), no warmup: every cast launch of the run is then one of the
  # S-image workload the bench's roofline leg times (always one pipeline), so the
  # kernel-stats average is comparable with roofline.avg_launch_us
  ARGS="--steps $S --warmup 0 --no-cpu-baseline --streams 1 ${PROF_ARGS:-}"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o trace -- \
      python3 "$ROOTDIR/bench.py" $ARGS > "$OUT/trace_bench.log" 2>&1
  rc=$?; echo "trace S=$S rc=$rc"; [ $rc -eq 0 ] || exit $rc
  if [ -n "${PMC:-}" ]; then
    for ctr in FETCH_SIZE WRITE_SIZE TCC_EA0_RDREQ_sum; do
      timeout -k 10 400 rocprofv3 --pmc $ctr --kernel-trace -f csv -d "$OUT" -o pmc_$ctr -- \
          python3 "$ROOTDIR/bench.py" $ARGS > "$OUT/pmc_${ctr}.log" 2>&1
      rc=$?; echo "pmc S=$S $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
  fi
done
if [ -z "${NO_DEFAULT_TRACE:-}" ]; then
  OUT="$ROOTDIR/gpurun_out/prof"
  mkdir -p "$OUT"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o trace_default -- \
      python3 "$ROOTDIR/bench.py" --no-cpu-baseline ${PROF_ARGS:-} > "$OUT/trace_default_bench.log" 2>&1
  rc=$?; echo "trace (default command) rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
