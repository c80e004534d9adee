#!/bin/bash
# MATERIAL's VALU lane utilisation (rocprofv3 PMC VALUUtilization, one pass per mode) on
# tools/material_probe.py's default and all-diffuse scenes (GPU box); output under gpurun_out/mat.
set -u
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOTDIR/gpurun_out/mat"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for mode in default diffuse; do
  timeout -k 10 300 rocprofv3 --pmc VALUUtilization --kernel-trace -f csv -d "$OUT" -o $mode -- \
      python3 "$ROOTDIR/tools/material_probe.py" $mode > "$OUT/$mode.log" 2>&1
  rc=$?; echo "$mode rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
