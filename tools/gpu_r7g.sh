set -o pipefail
# configs[1] lone query: scan priority mode (0/1/2) x tree rotation (0/1) on the product library
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
for i in 1 2; do
  for m in "0 0" "2 0" "0 1" "2 1" "1 1"; do
    set -- $m
    PIR_QUERY_SCAN_EVEN=$1 PIR_QUERY_TREE_ROT=$2 timeout -k 10 200 python -u tools/queue_time.py 20 1024 2 1 1 40 >> gpurun_out/r7g_c2_lone_modes.log 2>&1 || exit 1
  done
done && cat gpurun_out/r7g_c2_lone_modes.log
