set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_default.log | cut -c 1-200
rm -rf gpurun_out/prof_c2 gpurun_out/prof_c24 gpurun_out/prof_c5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python bench.py --no-cpu > gpurun_out/prof_c2.log 2>&1 || exit $?
tail -1 gpurun_out/prof_c2.log | cut -c 1-200
for c in c24 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- python bench.py --config $c --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_$c.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/bench_$c.log').read().strip().splitlines() if l.startswith('{')][-1]); print('$c', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'], d.get('roofline',{}).get('frac'))"
done
