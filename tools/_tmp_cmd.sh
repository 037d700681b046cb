set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
python -c "import json,sys; d=json.loads(open('gpurun_out/bench_default.log').read().strip().splitlines()[-1]); print('c2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'], d['roofline']['frac'], d['single_query']['ms_per_query'], d['parity'])"
for c in c24 c3 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_$c.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/bench_$c.log').read().strip().splitlines() if l.startswith('{')][-1]); print('$c', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'], d['roofline']['frac'], d['single_query']['ms_per_query'])"
done
timeout -k 10 300 python bench.py --config c3b --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_c3b.log 2>&1 || exit $?
python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/bench_c3b.log').read().strip().splitlines() if l.startswith('{')][-1]); print('c3b', d['value'], d['ms_per_step'])"
