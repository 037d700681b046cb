cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 100 python -c "
import sys; sys.argv=['x']; sys.path.insert(0,'tools'); import stream_probe as s
s.run(24, 256, 2, 1, 16); s.run(20, 1024, 2, 1, 50); s.run(24, 1024, 2, 1, 8); s.run(22, 128, 2, 1, 16)" || exit $?
timeout -k 10 120 python tools/trace_query.py --n 24 --efs 256 --reps 1 --queue 2 | tail -4 || exit $?
