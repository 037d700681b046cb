set -o pipefail
# configs[4]: the scan waves' ready poll (s_sleep 1 vs 16) -- does a waiting scan slow the tree?
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
ALT=$PWD/erasurecodedpir_amd/csrc/build_alt/libpir_engine_sleep16.so &&
for i in 1 2; do
  timeout -k 10 200 python -u tools/queue_time.py >> gpurun_out/r6l_c5_sleep_ab.log 2>&1 &&
  PIR_ENGINE_LIB=$ALT timeout -k 10 200 python -u tools/queue_time.py >> gpurun_out/r6l_c5_sleep_ab.log 2>&1 || exit 1
done &&
PIR_ENGINE_LIB=$ALT timeout -k 10 300 python -u tools/trace_query.py --n 24 --p 8 --nq 5 --queue 2 --reps 1 > gpurun_out/r6l_trace_c5_sleep16.log 2>&1 &&
cat gpurun_out/r6l_c5_sleep_ab.log && grep -h "queue tile\|shader clock between" gpurun_out/r6l_trace_c5_sleep16.log
