set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
timeout -k 10 400 python -u tools/fanout_probe.py 24 16 20 200 2000 > gpurun_out/r6e_fanout_new.log 2>&1 && cat gpurun_out/r6e_fanout_new.log &&
PIR_ENGINE_LIB=$PWD/erasurecodedpir_amd/csrc/build_alt/libpir_engine_oldshim.so timeout -k 10 400 python -u tools/fanout_probe.py 24 16 20 200 > gpurun_out/r6e_fanout_oldshim.log 2>&1 && cat gpurun_out/r6e_fanout_oldshim.log
