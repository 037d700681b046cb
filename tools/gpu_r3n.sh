# round 3: 2-rank rehearsal with HIP error logging (diagnose the n1_reference h2d failure)
set -o pipefail
mkdir -p gpurun_out
AMD_LOG_LEVEL=1 PIR_BENCH_REHEARSAL=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 4 --warmup 1 --no-cpu > gpurun_out/r3n_rehearsal_n2.log 2> gpurun_out/r3n_rehearsal_n2.err
echo "rc=$?" >> gpurun_out/r3n_rehearsal_n2.err
