#!/bin/bash
# rocprofv3 passes over a short bench run (GPU box). Kernel trace + stats first,
# then one PMC counter per pass (counters never combined with other traces).
set -u
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOTDIR/gpurun_out/prof"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
# Kernel summary of ONE pipeline (--streams 1), no warmup: every cast launch of the run is
# then one of the 64-image workload the bench's roofline leg times (always one pipeline),
# so the kernel-stats average is comparable with roofline.avg_launch_us. The default
# command (two concurrent pipelines, whose kernels overlap) is traced separately below.
ARGS="--steps ${PROF_STEPS:-64} --warmup 0 --no-cpu-baseline --streams 1 ${PROF_ARGS:-}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o trace -- \
    python3 "$ROOTDIR/bench.py" $ARGS > "$OUT/trace_bench.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o trace_default -- \
    python3 "$ROOTDIR/bench.py" --no-cpu-baseline ${PROF_ARGS:-} > "$OUT/trace_default_bench.log" 2>&1
rc=$?; echo "trace (default command) rc=$rc"; [ $rc -eq 0 ] || exit $rc
if [ -n "${PMC:-}" ]; then
  for ctr in FETCH_SIZE WRITE_SIZE TCC_EA0_RDREQ_sum; do
    timeout -k 10 400 rocprofv3 --pmc $ctr --kernel-trace -f csv -d "$OUT" -o pmc_$ctr -- \
        python3 "$ROOTDIR/bench.py" $ARGS \
        > "$OUT/pmc_${ctr}.log" 2>&1
    rc=$?; echo "pmc $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
fi
