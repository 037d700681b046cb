#!/bin/bash
# round 4, pass AE: 2-share sqrt(N) k_query with 4 share waves + 12 scan waves
# (libpir_engine_tw4.so): the cd / multiparty suites on it, then the cm A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PIR_ENGINE_LIB=$PWD/erasurecodedpir_amd/libpir_engine_tw4.so
timeout -k 10 400 python -u -m pytest tests/test_cd.py tests/test_multiparty.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r4ae_pytest.log 2>&1 || exit $?
run() {  # label env...
  echo "## $1" >> gpurun_out/r4ae_ab.jsonl
  env "${@:2}" timeout -k 10 300 python -u bench.py --config cm --steps 20 --warmup 3 --no-cpu \
    >> gpurun_out/r4ae_ab.jsonl 2>> gpurun_out/r4ae_ab.err
}
for rep in 1 2; do
  run two PIR_MP_FUSED=0 || exit $?
  run fused_tw4 PIR_MP_FUSED=2 || exit $?
  run fused_tw8 PIR_MP_FUSED=2 PIR_MP_TW=8 || exit $?
done
