# round 3: k_query reduce modes (0 = k_reduce, 1 = last workgroup, 2 = memory-side atomics)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fused_reduce or golden_answers or stream_equals" --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r3l_pytest.log 2>&1 || exit 1
for m in 0 2 1 2 0; do
PIR_FUSED_REDUCE=$m timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu --no-extras > gpurun_out/r3l_c2_fr$m.log 2>&1 || exit 2
cat gpurun_out/r3l_c2_fr$m.log >> gpurun_out/r3l_c2_all.log
done
for m in 0 2; do
PIR_FUSED_REDUCE=$m timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-extras > gpurun_out/r3l_c24_fr$m.log 2>&1 || exit 3
done
