cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 tests/test_gpu_parity.py -k "comm_path" > gpurun_out/pytest_comm.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_comm.log; [ $rc -eq 0 ] || exit $rc
CONFIGS="c2 c24" bash tools/gpu_profile.sh || exit $?
