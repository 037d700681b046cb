cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 tests/test_wire.py > gpurun_out/pytest_wire.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_wire.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/run_end_to_end.py > gpurun_out/e2e_c0.log 2>&1; rc=$?; tail -2 gpurun_out/e2e_c0.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/run_end_to_end.py --L 20 --f 1024 --k 5 --r 2 --down 2 > gpurun_out/e2e_k5.log 2>&1; rc=$?; tail -2 gpurun_out/e2e_k5.log; exit $rc
