# round 3: rehearsal matrix (ranks share this GPU): n=8 short, n=4 default, to localise the
# n1_reference h2d failure of the n=8 default run
set -o pipefail
mkdir -p gpurun_out
AMD_LOG_LEVEL=2 PIR_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29536 bench.py --gpus 8 --steps 4 --warmup 1 --no-cpu > gpurun_out/r3p_n8_short.log 2> gpurun_out/r3p_n8_short.err; echo "rc=$?" >> gpurun_out/r3p_n8_short.err
PIR_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29537 bench.py --gpus 4 > gpurun_out/r3p_n4.log 2> gpurun_out/r3p_n4.err; echo "rc=$?" >> gpurun_out/r3p_n4.err
