#!/bin/bash
# round 4, pass AB: k_query's XCD balance (libpir_engine_xb.so): its parity tests, the whole GPU
# suite on it, the per-XCD trace, then the bench A/B against the current library
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
XB=$PWD/erasurecodedpir_amd/libpir_engine_xb.so
PIR_ENGINE_LIB=$XB timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "xcd_balance" \
  --timeout 200 --timeout-method thread > gpurun_out/r4ab_pytest_xb.log 2>&1 || exit $?
PIR_ENGINE_LIB=$XB timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
  > gpurun_out/r4ab_pytest_all.log 2>&1 || exit $?
PIR_ENGINE_LIB=$XB timeout -k 10 120 python -u tools/trace_query.py --n 24 --reps 1 --queue 4 > gpurun_out/r4ab_trace_xb.txt 2>&1 || exit $?
run() {  # label config env...
  echo "## $1 $2" >> gpurun_out/r4ab_ab.jsonl
  env "${@:3}" timeout -k 10 300 python -u bench.py --config $2 --steps 20 --warmup 5 --no-cpu --no-extras \
    >> gpurun_out/r4ab_ab.jsonl 2>> gpurun_out/r4ab_ab.err
}
for rep in 1 2; do
  for c in c24 c5 c2 ccd; do
    run cur $c PIR_X=1 || exit $?
    run xb $c PIR_ENGINE_LIB=$XB || exit $?
  done
done
