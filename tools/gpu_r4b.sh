#!/bin/bash
# round 4, pass B: thread fan-out (C++ pool) + full-occupancy fold tests; configs[2] leaf-stage
# A/B (2-table AES at two workgroups per CU vs the 4-table stage); the default bench line; the
# hybrid AES micro-benchmark; then counters at HEAD (traffic, instruction mix, issue/wait
# breakdown, LDS) for c24, c5 and c3b, the library sha recorded beside each (tools/gpu_pmc.sh)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_threads.py tests/test_gpu_m4r_folds.py -x -v \
  --timeout 200 --timeout-method thread > gpurun_out/r4b_pytest.log 2>&1 || exit $?
for t2 in 1 0; do
  PIR_LEAF_T2=$t2 timeout -k 10 300 python -u bench.py --config c3b --steps 3 --warmup 1 \
    >> gpurun_out/r4b_c3b_t2.jsonl 2>&1 || exit $?
done
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4b_bench.json 2> gpurun_out/r4b_bench.err || exit $?
timeout -k 10 120 tools/micro/aes_hybrid > gpurun_out/r4b_aes_hybrid.txt 2>&1 || exit $?
timeout -k 10 120 tools/micro/aes_bitsliced > gpurun_out/r4b_aes_bitsliced.txt 2>&1 || exit $?
K=10 CONFIGS="c24 c5" PASSES="traffic insts active" tools/gpu_pmc.sh > gpurun_out/r4b_pmc.txt 2>&1 || exit $?
K=2 CONFIGS="c3b" PASSES="traffic insts active lds" tools/gpu_pmc.sh >> gpurun_out/r4b_pmc.txt 2>&1 || exit $?
