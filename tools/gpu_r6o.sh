set -o pipefail
# configs[4]: scan waves evened by priority ($PIR_QUERY_SCAN_EVEN=1) against the fixed priority
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
export PIR_ENGINE_LIB=$PWD/erasurecodedpir_amd/csrc/build_alt/libpir_engine_tt.so &&
for i in 1 2; do
  PIR_QUERY_SCAN_EVEN=0 timeout -k 10 200 python -u tools/queue_time.py >> gpurun_out/r6p_c5_even_ab.log 2>&1 &&
  PIR_QUERY_SCAN_EVEN=1 timeout -k 10 200 python -u tools/queue_time.py >> gpurun_out/r6p_c5_even_ab.log 2>&1 || exit 1
done &&
PIR_QUERY_SCAN_EVEN=2 PIR_TRACE_TILES=4,12 timeout -k 10 300 python -u tools/trace_query.py --n 24 --p 8 --nq 5 --queue 2 --reps 1 > gpurun_out/r6p_trace_c5_even.log 2>&1 &&
cat gpurun_out/r6p_c5_even_ab.log && grep -h -A1 "tree tile\|queue tile" gpurun_out/r6p_trace_c5_even.log
