set -o pipefail
# evened scan waves + rotated tree waves on the other k_query shapes (c24 queue, configs[1] lone,
# 256 B records queue, 3-4 round m4r queues): off (0,0) against on (2,1)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
export PIR_ENGINE_LIB=$PWD/erasurecodedpir_amd/csrc/build_alt/libpir_engine_tt.so &&
for shape in "24 1024 2 1 20 3" "20 1024 2 1 1 30" "24 256 2 1 20 3" "24 1024 4 3 20 3" "24 1024 5 4 20 3"; do
  for i in 1 2; do
    PIR_QUERY_SCAN_EVEN=0 PIR_QUERY_TREE_ROT=0 timeout -k 10 200 python -u tools/queue_time.py $shape >> gpurun_out/r6s_shapes_ab.log 2>&1 &&
    PIR_QUERY_SCAN_EVEN=2 PIR_QUERY_TREE_ROT=1 timeout -k 10 200 python -u tools/queue_time.py $shape >> gpurun_out/r6s_shapes_ab.log 2>&1 || exit 1
  done
done && cat gpurun_out/r6s_shapes_ab.log
