set -o pipefail
# configs[4]: tree waves rotated over the narrow levels tile by tile ($PIR_QUERY_TREE_ROT=1) on
# top of the SIMD-mate scan priority ($PIR_QUERY_SCAN_EVEN=2); parity of both on the m4r tests
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
export PIR_ENGINE_LIB=$PWD/erasurecodedpir_amd/csrc/build_alt/libpir_engine_tt.so &&
PIR_QUERY_SCAN_EVEN=2 PIR_QUERY_TREE_ROT=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_m4r_folds.py tests/test_gpu_parity.py -k "m4r or query" > gpurun_out/r6q_pytest.log 2>&1 &&
tail -3 gpurun_out/r6q_pytest.log &&
for i in 1 2; do
  PIR_QUERY_SCAN_EVEN=0 timeout -k 10 200 python -u tools/queue_time.py >> gpurun_out/r6q_c5_ab.log 2>&1 &&
  PIR_QUERY_SCAN_EVEN=2 timeout -k 10 200 python -u tools/queue_time.py >> gpurun_out/r6q_c5_ab.log 2>&1 &&
  PIR_QUERY_SCAN_EVEN=2 PIR_QUERY_TREE_ROT=1 timeout -k 10 200 python -u tools/queue_time.py >> gpurun_out/r6q_c5_ab.log 2>&1 &&
  PIR_QUERY_SCAN_EVEN=0 PIR_QUERY_TREE_ROT=1 timeout -k 10 200 python -u tools/queue_time.py >> gpurun_out/r6q_c5_ab.log 2>&1 || exit 1
done &&
PIR_QUERY_SCAN_EVEN=2 PIR_QUERY_TREE_ROT=1 PIR_TRACE_TILES=4,12 timeout -k 10 300 python -u tools/trace_query.py --n 24 --p 8 --nq 5 --queue 2 --reps 1 > gpurun_out/r6q_trace_c5.log 2>&1 &&
cat gpurun_out/r6q_c5_ab.log && grep -h -A1 "tree tile\|queue tile" gpurun_out/r6q_trace_c5.log
