# round 3: 5-round scans -- k_scan_t forced vs the 768-thread GPR-index k_scan_uni (Hollanti, 1 KiB)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --config ch5 --steps 5 --warmup 2 --no-cpu --no-extras > gpurun_out/r3j_ch5_uni.log 2>&1 || exit 1
PIR_SCAN_T=2 timeout -k 10 200 python bench.py --config ch5 --steps 5 --warmup 2 --no-cpu --no-extras > gpurun_out/r3j_ch5_t.log 2>&1 || exit 2
PIR_SCAN_T=2 timeout -k 10 300 python -u -m pytest tests/test_hollanti.py tests/test_multiparty.py tests/test_gpu_batch.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r3j_pytest_t2.log 2>&1 || exit 3
