#!/bin/bash
# round 4, pass X: k_query's tail help (a lone query's tree waves fold half of the last tile),
# built as libpir_engine_tail.so: its parity tests, the whole GPU suite on it, then the lone-query
# A/B (configs[1] and north_star single) against the current library and PIR_QUERY_TAIL=0
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TL=$PWD/erasurecodedpir_amd/libpir_engine_tail.so
PIR_ENGINE_LIB=$TL timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "tail_help" \
  --timeout 200 --timeout-method thread > gpurun_out/r4x_pytest_tail.log 2>&1 || exit $?
PIR_ENGINE_LIB=$TL timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
  > gpurun_out/r4x_pytest_all.log 2>&1 || exit $?
run() {  # label config env...
  echo "## $1 $2" >> gpurun_out/r4x_ab.jsonl
  env "${@:3}" timeout -k 10 300 python -u bench.py --config $2 --steps 50 --warmup 5 --no-cpu --no-extras \
    >> gpurun_out/r4x_ab.jsonl 2>> gpurun_out/r4x_ab.err
}
for rep in 1 2; do
  for c in c2 c24; do
    run cur $c PIR_X=1 || exit $?
    run tail $c PIR_ENGINE_LIB=$TL || exit $?
    run tail_off $c PIR_ENGINE_LIB=$TL PIR_QUERY_TAIL=0 || exit $?
  done
done
