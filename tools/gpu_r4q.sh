#!/bin/bash
# round 4, pass Q: defaults after the sqrt(N) k_query rule (>= 3 shares), and the share waves'
# priority in that mode (3, the lone-query default, vs 0)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cd.py tests/test_multiparty.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r4q_pytest.log 2>&1 || exit $?
run() {  # config, label, env...
  echo "## $1 $2 ${*:3}" >> gpurun_out/r4q_ab.jsonl
  env "${@:3}" timeout -k 10 300 python -u bench.py --config $1 --steps 20 --warmup 3 \
    >> gpurun_out/r4q_ab.jsonl 2>> gpurun_out/r4q_ab.err
}
for rep in 1 2; do
  for c in ccd ccd7; do
    run $c prio3 PIR_QUERY_TREE_PRIO=3 || exit $?
    run $c prio0 PIR_QUERY_TREE_PRIO=0 || exit $?
    run $c prio1 PIR_QUERY_TREE_PRIO=1 || exit $?
  done
  run cm default PIR_X=1 || exit $?
done
