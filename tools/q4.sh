cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 tests/test_gpu_parity.py -k "stream or fused_path" > gpurun_out/pytest_q4.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_q4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python -c "
import sys; sys.argv=['x']; sys.path.insert(0,'tools'); import stream_probe as s
s.run(24, 256, 2, 1, 16); s.run(22, 256, 2, 1, 16); s.run(24, 128, 2, 1, 16)" || exit $?
PIR_QUERY_TW=8 timeout -k 10 100 python -c "
import sys; sys.argv=['x']; sys.path.insert(0,'tools'); import stream_probe as s
s.run(24, 256, 2, 1, 16); s.run(22, 256, 2, 1, 16); s.run(24, 128, 2, 1, 16)" || exit $?
