set -o pipefail
# the N > 1 path rehearsed on one GPU at the final library: 8 ranks sharing the card, host gloo
# fold (PIR_BENCH_REHEARSAL=1), then N = 2
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
PIR_BENCH_REHEARSAL=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 8 > gpurun_out/r7h_rehearsal_n8.jsonl 2> gpurun_out/r7h_rehearsal_n8.err &&
PIR_BENCH_REHEARSAL=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 > gpurun_out/r7h_rehearsal_n2.jsonl 2> gpurun_out/r7h_rehearsal_n2.err &&
tail -c 700 gpurun_out/r7h_rehearsal_n8.jsonl && tail -c 400 gpurun_out/r7h_rehearsal_n2.jsonl
