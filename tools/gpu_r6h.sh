set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
timeout -k 10 120 tools/micro/aes_col_latency > gpurun_out/r6h_aes_col_latency.log 2>&1; cat gpurun_out/r6h_aes_col_latency.log &&
timeout -k 10 300 python -u tools/trace_query.py --n 20 --reps 2 > gpurun_out/r6h_trace_c2.log 2>&1 && cat gpurun_out/r6h_trace_c2.log
