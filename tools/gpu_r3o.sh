# round 3: 8-rank rehearsal with HIP error logging (ranks share this GPU; default steps/warmup)
set -o pipefail
mkdir -p gpurun_out
t0=$SECONDS
AMD_LOG_LEVEL=1 PIR_BENCH_REHEARSAL=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 8 > gpurun_out/r3o_rehearsal_n8.log 2> gpurun_out/r3o_rehearsal_n8.err
echo "rc=$? wall $((SECONDS - t0))s" >> gpurun_out/r3o_rehearsal_n8.err
