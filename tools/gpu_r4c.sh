#!/bin/bash
# round 4, pass C: fan-out without the server-lock convoy (threads tests), the guard-free
# four-Russians k_query loads (parity: folds at full occupancy, m4r == plane masks, the
# configs[4] libref golden), the default bench line, then counters at HEAD for c24, c5, c3b
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_threads.py tests/test_gpu_m4r_folds.py \
  tests/test_gpu_parity.py -k "threads or m4r or concurrent or slices" -x -v \
  --timeout 200 --timeout-method thread > gpurun_out/r4c_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest "tests/test_gpu_fullsize.py::test_fullsize24_golden_query" -x -v \
  --timeout 250 --timeout-method thread >> gpurun_out/r4c_pytest.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4c_bench.json 2> gpurun_out/r4c_bench.err || exit $?
K=10 CONFIGS="c24 c5" PASSES="traffic insts active" tools/gpu_pmc.sh > gpurun_out/r4c_pmc.txt 2>&1 || exit $?
K=2 CONFIGS="c3b" PASSES="traffic insts active lds" tools/gpu_pmc.sh >> gpurun_out/r4c_pmc.txt 2>&1 || exit $?
