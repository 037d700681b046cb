set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
timeout -k 10 300 tools/micro/fold_mix > gpurun_out/r6b_fold_mix.log 2>&1 && cat gpurun_out/r6b_fold_mix.log &&
timeout -k 10 120 tools/micro/aes_sbox_latency > gpurun_out/r6b_sbox.log 2>&1; rc=$?; cat gpurun_out/r6b_sbox.log; [ $rc -le 2 ] &&
tools/gpu_steps.sh r6b sha bench &&
PIR_BENCH_REHEARSAL=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 8 > gpurun_out/r6b_rehearsal_n8.jsonl 2> gpurun_out/r6b_rehearsal_n8.err && tail -c 600 gpurun_out/r6b_rehearsal_n8.jsonl
