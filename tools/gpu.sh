#!/bin/bash
# gpurun wrapper: re-submit only when the GPU service reports an infrastructure event
# ("status=transient": nothing ran, nothing charged).  Any other outcome is returned as is.
# usage: tools/gpu.sh TIMEOUT_S 'command'
to=$1; shift
for attempt in 1 2 3 4; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$to" -- "$@" 2>&1)
  rc=$?
  if echo "$out" | grep -q "status=transient"; then
    echo "[gpu.sh] transient (attempt $attempt), waiting"; sleep 60; continue
  fi
  echo "$out"
  exit $rc
done
echo "$out"; exit $rc
