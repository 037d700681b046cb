# round 3: byte-trimmed leaf blocks in k_query / k_expand / k_fused: parity, then a same-box A/B
# against the previous build (tools/_tmp_ab/libpir_engine_head.so) on the tree-bound shapes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r3u_pytest.log 2>&1 || exit 1
for v in new head new head; do
  if [ $v = head ]; then export PIR_ENGINE_LIB=$GRAFT_REPO_ROOT/tools/_tmp_ab/libpir_engine_head.so; else unset PIR_ENGINE_LIB; fi
  timeout -k 10 200 python bench.py --config c3 --steps 10 --warmup 3 --no-cpu --no-extras >> gpurun_out/r3u_c3_$v.log 2>&1 || exit 2
  timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu --no-extras >> gpurun_out/r3u_c2_$v.log 2>&1 || exit 3
done
