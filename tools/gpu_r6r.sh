set -o pipefail
# configs[4] with evened scan waves + rotated tree waves: the tree waves' priority (3 = current)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
export PIR_ENGINE_LIB=$PWD/erasurecodedpir_amd/csrc/build_alt/libpir_engine_tt.so PIR_QUERY_SCAN_EVEN=2 PIR_QUERY_TREE_ROT=1 &&
for i in 1 2; do
  for tp in 3 2 1 0; do
    PIR_QUERY_TREE_PRIO=$tp timeout -k 10 200 python -u tools/queue_time.py >> gpurun_out/r6r_c5_tprio.log 2>&1 || exit 1
  done
done &&
PIR_QUERY_TREE_PRIO=1 PIR_TRACE_TILES=4,12 timeout -k 10 300 python -u tools/trace_query.py --n 24 --p 8 --nq 5 --queue 2 --reps 1 > gpurun_out/r6r_trace_c5_tp1.log 2>&1 &&
cat gpurun_out/r6r_c5_tprio.log && grep -h -A1 "tree tile\|queue tile" gpurun_out/r6r_trace_c5_tp1.log
