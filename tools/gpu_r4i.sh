#!/bin/bash
# round 4, pass I: pir_comm_detach on the 1-rank communicator, and the bench's host-fold
# exchange (rehearsal: 2 ranks sharing the GPU, partition answers XORed over gloo inside the
# timed region -- the path an RCCL-init failure now falls back to)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "comm_path" \
  --timeout 120 --timeout-method thread > gpurun_out/r4i_pytest.log 2>&1 || exit $?
PIR_BENCH_REHEARSAL=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 \
  --warmup 3 > gpurun_out/r4i_rehearsal_n2.json 2> gpurun_out/r4i_rehearsal_n2.err
