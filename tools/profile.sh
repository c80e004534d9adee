#!/bin/bash
# rocprofv3 passes over a short bench run (GPU box). Kernel trace + stats first,
# then one PMC counter per pass (counters never combined with other traces).
set -u
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOTDIR/gpurun_out/prof"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ARGS="--steps ${PROF_STEPS:-16} --warmup 1 --roofline-images 2 --no-cpu-baseline ${PROF_ARGS:-}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o trace -- \
    python3 "$ROOTDIR/bench.py" $ARGS > "$OUT/trace_bench.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
if [ -n "${PMC:-}" ]; then
  for ctr in FETCH_SIZE WRITE_SIZE TCC_EA0_RDREQ_sum; do
    timeout -k 10 400 rocprofv3 --pmc $ctr --kernel-trace -f csv -d "$OUT" -o pmc_$ctr -- \
        python3 "$ROOTDIR/bench.py" --steps 2 --warmup 1 --roofline-images 1 --no-cpu-baseline ${PROF_ARGS:-} \
        > "$OUT/pmc_${ctr}.log" 2>&1
    rc=$?; echo "pmc $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
fi
