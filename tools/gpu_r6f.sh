set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
timeout -k 10 400 python -u tools/fanout_probe.py 24 16 20 > gpurun_out/r6f_fanout.log 2>&1 && cat gpurun_out/r6f_fanout.log &&
tools/gpu_steps.sh r6f pytest:tests/test_gpu_threads.py bench
