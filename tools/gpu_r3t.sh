# round 3 evidence: kernel trace + stats of the default bench command (no CPU leg)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3t_prof -o default --output-format csv -- python3 bench.py --no-cpu > gpurun_out/r3t_default.log 2>&1 || exit 1
