set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
{ timeout -k 10 120 tools/micro/aes_sbox_latency > gpurun_out/r6c_sbox.log 2>&1; rc=$?; cat gpurun_out/r6c_sbox.log; [ $rc -le 2 ]; } &&
timeout -k 10 300 python -u tools/free_probe.py 24 1 0 > gpurun_out/r6c_free_probe.log 2>&1 && cat gpurun_out/r6c_free_probe.log &&
tools/gpu_steps.sh r6c sha pytest smoke bench
