# round 3: pipelined k_scan_t lookups, 256-thread blocks x 4 (or 3) per CU: parity + c3b + ch5 (scan_t forced)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_batch.py tests/test_hollanti.py tests/test_multiparty.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r3h_pytest.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config c3b --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/r3h_c3b.log 2>&1 || exit 2
PIR_SCAN_T_BPC=3 timeout -k 10 200 python bench.py --config c3b --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/r3h_c3b_bpc3.log 2>&1 || exit 3
timeout -k 10 200 python bench.py --config cm4 --steps 5 --warmup 2 --no-cpu --no-extras > gpurun_out/r3h_cm4.log 2>&1 || exit 4
