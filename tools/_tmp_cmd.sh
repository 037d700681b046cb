set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_default.log | cut -c 1-400
for c in c5 c24 c3; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_$c.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_$c.log').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'))"
done
