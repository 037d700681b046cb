set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
for c in c3 c3b; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_$c.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/bench_$c.log').read().strip().splitlines() if l.startswith('{')][-1]); print('$c', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'), d.get('parity'))"
done
