set -o pipefail
# configs[4] (evened scan + rotated tree): the tree waves' priority lowered while the slowest scan
# wave still has two tiles to fold ($PIR_QUERY_TREE_DYN = 1: to 1, 2: to 2, 3: to 0; 0 = fixed 3)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
export PIR_ENGINE_LIB=$PWD/erasurecodedpir_amd/csrc/build_alt/libpir_engine_tt.so PIR_QUERY_SCAN_EVEN=2 PIR_QUERY_TREE_ROT=1 &&
for i in 1 2; do
  for td in 0 1 2 3; do
    PIR_QUERY_TREE_DYN=$td timeout -k 10 200 python -u tools/queue_time.py >> gpurun_out/r6t_c5_tdyn.log 2>&1 || exit 1
  done
done &&
for td in 0 1; do
  PIR_QUERY_TREE_DYN=$td timeout -k 10 200 python -u tools/queue_time.py 20 1024 2 1 1 30 >> gpurun_out/r6t_c5_tdyn.log 2>&1 || exit 1
done && cat gpurun_out/r6t_c5_tdyn.log
