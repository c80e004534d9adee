#!/bin/bash
# retry gpurun only while it reports "no slot/box free" (exit 3: nothing ran, nothing charged)
log=$1; shift
for attempt in $(seq 1 12); do
  /usr/local/graft/bin/gpurun "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -ne 3 ]; then exit $rc; fi
  sleep 120
done
exit 3
