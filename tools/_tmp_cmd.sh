set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_batch.py -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for B in 1 2; do for G in 8 16; do PIR_BATCH_SCAN_BPC=$B PIR_BATCH_G=$G timeout -k 10 300 python bench.py --config c3b --steps 2 --warmup 1 > gpurun_out/c3b_g$G.log 2>&1 || exit $?; echo "bpc=$B G=$G"; tail -1 gpurun_out/c3b_g$G.log | cut -c 180-300; done; done
rm -rf gpurun_out/prof_c3b
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3b -o run --output-format csv -- python bench.py --config c3b --steps 1 --warmup 1 > gpurun_out/prof_c3b.log 2>&1; echo rc=$?
