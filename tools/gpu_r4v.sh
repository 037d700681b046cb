#!/bin/bash
# round 4, pass V: the north_star single query (one launch per query, 4096-leaf tiles) against
# the lone-query tree priority (3 by default for nk == 1) and the queue
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() {  # label, env...
  echo "## $*" >> gpurun_out/r4v_c24.jsonl
  env "${@:2}" timeout -k 10 300 python -u bench.py --config c24 --steps 20 --warmup 5 --no-cpu --no-extras \
    >> gpurun_out/r4v_c24.jsonl 2>> gpurun_out/r4v_c24.err
}
for rep in 1 2; do
  run default PIR_X=1 || exit $?
  run prio0 PIR_QUERY_TREE_PRIO=0 || exit $?
  run prio1 PIR_QUERY_TREE_PRIO=1 || exit $?
done
