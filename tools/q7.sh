cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 tests/test_gpu_parity.py -k "stream or query or fused or slices or partition or full_size or comm" > gpurun_out/pytest_q7.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_q7.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python -c "
import sys; sys.argv=['x']; sys.path.insert(0,'tools'); import stream_probe as s
s.run(24, 256, 2, 1, 16); s.run(20, 1024, 2, 1, 50); s.run(24, 1024, 2, 1, 8); s.run(24, 1024, 8, 5, 4)" || exit $?
timeout -k 10 120 python tools/trace_query.py --n 24 --efs 256 --reps 1 --queue 2 | tail -6 || exit $?
timeout -k 10 120 python tools/trace_query.py --reps 1 | head -12 || exit $?
