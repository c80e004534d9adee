#!/bin/bash
# Run GPU steps in order on the box; each step has its own time limit. A step that ends
# in a fault / abort / segfault / time limit (rc 124, 134, 137, 139 or any > 128) stops
# the call: nothing more touches the GPU. Ordinary failures (rc 1, e.g. a failed test)
# are recorded and the next step runs.
#   tools/gpu_steps.sh "SECONDS:command" ["SECONDS:command" ...]
set -u
mkdir -p gpurun_out
for step in "$@"; do
  secs=${step%%:*}; cmd=${step#*:}
  echo "[step] $cmd (limit ${secs}s)"
  timeout -k 10 "$secs" bash -c "$cmd"
  rc=$?
  echo "[step] rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "[step] stopping: fault/abort/time limit"; exit $rc; fi
done
