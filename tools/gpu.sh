#!/bin/bash
# gpurun wrapper: re-submit only when the GPU service reports an infrastructure event
# ("status=transient": nothing ran, nothing charged) or no free box (exit 3).  Any other
# outcome is returned as is.
# usage: tools/gpu.sh TIMEOUT_S 'command'
to=$1; shift
for attempt in $(seq 1 30); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$to" -- "$@" 2>&1)
  rc=$?
  if echo "$out" | grep -q "status=transient" || [ $rc -eq 3 ]; then
    echo "[gpu.sh] transient/no box (attempt $attempt), waiting"; sleep 90; continue
  fi
  echo "$out"
  exit $rc
done
echo "$out"; exit $rc
