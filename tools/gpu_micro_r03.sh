#!/bin/bash
# Round-3 micro-benchmarks + the batched configs[2] kernel trace.  Every GPU step time-limited;
# a failure ends the session.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03_micro
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/r03_micro/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 12 "gpurun_out/r03_micro/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
for m in ${MICROS:-aes_bitsliced aes_latency aes_node}; do step $m 120 tools/micro/$m; done
if [ -n "$PROF_CFG" ]; then
  rm -rf gpurun_out/prof_$PROF_CFG
  step prof_$PROF_CFG 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$PROF_CFG -o run --output-format csv -- python bench.py --config $PROF_CFG --steps 3 --warmup 1 --no-cpu --no-extras
fi
exit 0
