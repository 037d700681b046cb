set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_batch.py -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c3b --steps 2 --warmup 1 > gpurun_out/c3b.log 2>&1 || exit $?; tail -1 gpurun_out/c3b.log | cut -c 180-700
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu > gpurun_out/c2.log 2>&1 || exit $?; tail -1 gpurun_out/c2.log | cut -c 1-300
rm -rf gpurun_out/prof_c3b
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3b -o run --output-format csv -- python bench.py --config c3b --steps 1 --warmup 1 > gpurun_out/prof_c3b.log 2>&1; echo rc=$?
