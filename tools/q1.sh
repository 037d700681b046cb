# quick GPU check of the single-launch query path: parity subset, phase trace, c2/c24 bench
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 tests/test_gpu_parity.py -k "fused or query or full_size or multi_round or slices or partition" > gpurun_out/pytest_q.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_q.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/trace_query.py --reps 1 || exit $?
timeout -k 10 120 python tools/trace_query.py --n 24 --reps 1 || exit $?
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu > gpurun_out/bench_c2.log 2>&1 || exit $?; tail -1 gpurun_out/bench_c2.log | cut -c 1-900
timeout -k 10 300 python bench.py --config c24 --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_c24.log 2>&1 || exit $?; tail -1 gpurun_out/bench_c24.log | cut -c 1-900
