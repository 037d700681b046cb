#!/bin/bash
# round 4, first GPU pass: thread-call shape + key-major batch parity + in-kernel reduce modes,
# then the driver bench and same-box A/Bs (configs[2] key-major packed shares vs interleaved;
# configs[1] lone query with k_reduce vs the per-XCD in-kernel reduce)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_threads.py tests/test_gpu_batch.py \
  "tests/test_gpu_parity.py::test_fused_reduce_equals_k_reduce" -x -v \
  --timeout 200 --timeout-method thread > gpurun_out/r4a_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config c3b --steps 3 --warmup 1 > gpurun_out/r4a_c3b_new.json 2>&1 || exit $?
PIR_BATCH_KMAJOR=0 PIR_LEAF_PACK=0 timeout -k 10 300 python -u bench.py --config c3b --steps 3 --warmup 1 \
  > gpurun_out/r4a_c3b_old.json 2>&1 || exit $?
for fr in 0 3 0 3; do
  PIR_FUSED_REDUCE=$fr timeout -k 10 300 python -u bench.py --config c2 --steps 20 --warmup 5 --no-cpu --no-extras \
    >> gpurun_out/r4a_c2_reduce.jsonl 2>&1 || exit $?
done
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4a_bench.json 2> gpurun_out/r4a_bench.err
