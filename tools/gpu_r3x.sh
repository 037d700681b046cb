# round 3: packed four-Russians indices, extracts 3 planes ahead (tools/gen_m4r.py).  The 4-round
# test that took stale indices, with and without an s_nop after every index change
# (tools/_tmp_ab/libpir_engine_wait.so); then the whole GPU suite and a same-box A/B against the
# unpacked fold (tools/_tmp_ab/libpir_engine.so) with the variant that passed.
set -o pipefail
mkdir -p gpurun_out
T='tests/test_gpu_encode.py::test_configs4_pipeline_end_to_end'
A=$GRAFT_REPO_ROOT/tools/_tmp_ab
timeout -k 10 120 python -u -m pytest "$T" -m gpu -q --timeout 60 --timeout-method thread -p no:cacheprovider > gpurun_out/r3x_new.log 2>&1
rn=$?; echo "new rc=$rn"
PIR_ENGINE_LIB=$A/libpir_engine_wait.so timeout -k 10 120 python -u -m pytest "$T" -m gpu -q --timeout 60 --timeout-method thread -p no:cacheprovider > gpurun_out/r3x_wait.log 2>&1
rw=$?; echo "wait rc=$rw"
if [ $rn = 0 ]; then unset PIR_ENGINE_LIB; NEW=""; elif [ $rw = 0 ]; then NEW=$A/libpir_engine_wait.so; else exit 1; fi
echo "suite with '${NEW:-in-tree}'"
PIR_ENGINE_LIB=$NEW timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r3x_pytest.log 2>&1 || exit 2
for v in new old new old; do
  if [ $v = old ]; then L=$A/libpir_engine.so; else L=$NEW; fi
  PIR_ENGINE_LIB=$L timeout -k 10 200 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu --no-extras >> gpurun_out/r3x_c5_$v.log 2>&1 || exit 3
  PIR_ENGINE_LIB=$L timeout -k 10 200 python bench.py --config ch5 --steps 10 --warmup 3 --no-cpu --no-extras >> gpurun_out/r3x_ch5_$v.log 2>&1 || exit 4
done
