# round 3: transposed four-Russians scan (k_scan_t): parity + c3b + Hollanti 5 rounds + multiparty
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_batch.py tests/test_hollanti.py tests/test_multiparty.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r3f_pytest.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config c3b --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/r3f_c3b.log 2>&1 || exit 2
PIR_BATCH_KLAST=5 timeout -k 10 200 python bench.py --config c3b --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/r3f_c3b_k5.log 2>&1 || exit 3
timeout -k 10 200 python bench.py --config ch5 --steps 5 --warmup 2 --no-cpu --no-extras > gpurun_out/r3f_ch5.log 2>&1 || exit 4
PIR_SCAN_T=0 timeout -k 10 200 python bench.py --config ch5 --steps 5 --warmup 2 --no-cpu --no-extras > gpurun_out/r3f_ch5_uni.log 2>&1 || exit 5
timeout -k 10 200 python bench.py --config cm4 --steps 5 --warmup 2 --no-cpu --no-extras > gpurun_out/r3f_cm4.log 2>&1 || exit 6
