# round 3: full -m gpu suite at HEAD, then the 8-rank rehearsal of bench.py --gpus 8 (ranks share
# this GPU, no RCCL; timing meaningless, wall time recorded against the driver's limit)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider --durations=5 > gpurun_out/r3m_pytest.log 2>&1 || exit 1
t0=$SECONDS
PIR_BENCH_REHEARSAL=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 > gpurun_out/r3m_rehearsal_n8.log 2> gpurun_out/r3m_rehearsal_n8.err || exit 2
echo "rehearsal wall ${SECONDS}s total, $((SECONDS - t0))s for bench.py --gpus 8 (default steps/warmup)" > gpurun_out/r3m_rehearsal_wall.txt
