# c5 scan check: parity for multi-round shapes, then trace + probe for p=8 NQ=5
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 tests/test_gpu_parity.py -k "nq5 or nq4 or nq3 or nq8 or multi_round or stream" > gpurun_out/pytest_q3.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_q3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/trace_query.py --n 24 --p 8 --nq 5 --reps 1 --queue 4 || exit $?
timeout -k 10 200 python bench.py --config c5 --steps 4 --warmup 1 --no-cpu > gpurun_out/bench_c5.log 2>&1; rc=$?; tail -1 gpurun_out/bench_c5.log | cut -c 1-700; exit $rc
