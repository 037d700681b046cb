# round 3: rehearsals after the n1_reference key-count fix (ranks share this GPU, default steps)
set -o pipefail
mkdir -p gpurun_out
t0=$SECONDS
PIR_BENCH_REHEARSAL=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29538 bench.py --gpus 8 > gpurun_out/r3q_rehearsal_n8.log 2> gpurun_out/r3q_rehearsal_n8.err || exit 1
echo "bench.py --gpus 8 (8 ranks on one GPU, default --steps 20 --warmup 5, incl. the CPU baseline leg of rank 0 and the 1-GPU 128 GiB reference): $((SECONDS - t0)) s wall" > gpurun_out/r3q_rehearsal_wall.txt
t0=$SECONDS
PIR_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29539 bench.py --gpus 4 > gpurun_out/r3q_rehearsal_n4.log 2> gpurun_out/r3q_rehearsal_n4.err || exit 2
echo "bench.py --gpus 4: $((SECONDS - t0)) s wall" >> gpurun_out/r3q_rehearsal_wall.txt
