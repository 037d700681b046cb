# round 3: depth-first node stages + shallow batched frontier: parity, c3b, kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r3d_pytest.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config c3b --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/r3d_c3b.log 2>&1 || exit 2
PIR_BATCH_KLAST=5 timeout -k 10 200 python bench.py --config c3b --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/r3d_c3b_k5.log 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3d_prof -o c3b --output-format csv -- python3 bench.py --config c3b --steps 2 --warmup 1 --no-cpu --no-extras > gpurun_out/r3d_c3b_prof.log 2>&1 || exit 4
# configs[4] k_query: tree-only (scan waves skip their rows) vs full, queue of 4
timeout -k 10 200 python tools/trace_query.py --n 24 --efs 1024 --p 8 --nq 5 --queue 4 --reps 1 > gpurun_out/r3d_c5_trace.log 2>&1 || exit 5
PIR_TRACE_NOSCAN=1 timeout -k 10 200 python tools/trace_query.py --n 24 --efs 1024 --p 8 --nq 5 --queue 4 --reps 1 > gpurun_out/r3d_c5_trace_noscan.log 2>&1 || exit 6
