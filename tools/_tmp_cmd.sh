set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
PIR_QUERY_TW=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fused or query or stream or multi_round or random_shapes or property" > gpurun_out/pytest_tw4.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_tw4.log; [ $rc -eq 0 ] || exit $rc
for tw in 8 4; do
  PIR_QUERY_TW=$tw timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_c5_tw$tw.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/bench_c5_tw$tw.log').read().strip().splitlines() if l.startswith('{')][-1]); print('c5 tw$tw', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'], d['roofline']['frac'], d['single_query']['ms_per_query'], d['parity'])"
done
