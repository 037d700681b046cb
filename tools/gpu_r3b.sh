# round 3: parity of the depth-first 4-table leaf stage + configs[2] batched A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r3b_pytest.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config c3b --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/r3b_c3b_dfs4.log 2>&1 || exit 2
PIR_BATCH_KLAST=5 timeout -k 10 200 python bench.py --config c3b --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/r3b_c3b_dfs4_k5.log 2>&1 || exit 3
PIR_LEAF_DFS=0 timeout -k 10 200 python bench.py --config c3b --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/r3b_c3b_bfs.log 2>&1 || exit 4
