#!/bin/bash
# round 4, pass J: tree ILP A/B (k_query tree waves: 2 nodes per lane in flight on the wide
# levels, PIR_TREE_ILP=2: libpir_engine_ilp2.so, against the one-chain default build), parity of
# the ILP build (the gpu tests that pin k_query, run against it)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
ILP2=$PWD/erasurecodedpir_amd/libpir_engine_ilp2.so
PIR_ENGINE_LIB=$ILP2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_threads.py -m gpu -x -q \
  --timeout 250 --timeout-method thread > gpurun_out/r4j_pytest.log 2>&1 || exit $?
for lib in ilp1 ilp2 ilp1 ilp2; do
  if [ $lib = ilp2 ]; then export PIR_ENGINE_LIB=$ILP2; else unset PIR_ENGINE_LIB; fi
  echo "## $lib" >> gpurun_out/r4j_ab.jsonl
  timeout -k 10 400 python -u bench.py --no-cpu >> gpurun_out/r4j_ab.jsonl 2>> gpurun_out/r4j_ab.err || exit $?
done
unset PIR_ENGINE_LIB
