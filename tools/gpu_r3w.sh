# diagnose test_configs4_pipeline_end_to_end[17-512-4-3] under the packed fold
set -o pipefail
mkdir -p gpurun_out
T='tests/test_gpu_encode.py::test_configs4_pipeline_end_to_end'
timeout -k 10 120 python -u -m pytest "$T" -m gpu -q --timeout 60 --timeout-method thread -p no:cacheprovider > gpurun_out/r3w_packed.log 2>&1
echo "packed rc=$?"
PIR_ENGINE_LIB=$GRAFT_REPO_ROOT/tools/_tmp_ab/libpir_engine.so timeout -k 10 120 python -u -m pytest "$T" -m gpu -q --timeout 60 --timeout-method thread -p no:cacheprovider > gpurun_out/r3w_unpacked.log 2>&1
echo "unpacked rc=$?"
PIR_QUERY_M4R=0 timeout -k 10 120 python -u -m pytest "$T" -m gpu -q --timeout 60 --timeout-method thread -p no:cacheprovider > gpurun_out/r3w_masks.log 2>&1
echo "masks rc=$?"
PIR_QUERY=0 timeout -k 10 120 python -u -m pytest "$T" -m gpu -q --timeout 60 --timeout-method thread -p no:cacheprovider > gpurun_out/r3w_unfused.log 2>&1
echo "unfused rc=$?"
exit 0
