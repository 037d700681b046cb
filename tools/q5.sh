cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 tests/test_gpu_encode.py > gpurun_out/pytest_enc.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_enc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/c5_e2e.py > gpurun_out/c5_e2e.log 2>&1; rc=$?; tail -3 gpurun_out/c5_e2e.log; exit $rc
