#!/bin/bash
# round 4, pass AC: which block parity the XCD balance should favour -- per-XCD trace and the
# north_star queue with the balance forced (PIR_XCD_BALANCE 0 / 1 / 2) on libpir_engine_xb.so
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PIR_ENGINE_LIB=$PWD/erasurecodedpir_amd/libpir_engine_xb.so
for xb in 0 1 2; do
  echo "## balance $xb" >> gpurun_out/r4ac_trace.txt
  PIR_XCD_BALANCE=$xb timeout -k 10 120 python -u tools/trace_query.py --n 24 --reps 1 --queue 4 >> gpurun_out/r4ac_trace.txt 2>&1 || exit $?
done
for rep in 1 2; do
  for xb in 0 1 2 d; do
    echo "## balance $xb" >> gpurun_out/r4ac_ab.jsonl
    if [ $xb = d ]; then unset PIR_XCD_BALANCE; else export PIR_XCD_BALANCE=$xb; fi
    timeout -k 10 300 python -u bench.py --config c24 --steps 20 --warmup 5 --no-cpu --no-extras \
      >> gpurun_out/r4ac_ab.jsonl 2>> gpurun_out/r4ac_ab.err || exit $?
  done
done
