#!/bin/bash
# round 4, pass T: configs[1] lone query -- first-tile size and tree-wave priority re-measured on
# the final library (ILP tree)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() {  # label, env...
  echo "## $*" >> gpurun_out/r4t_c2.jsonl
  env "${@:2}" timeout -k 10 300 python -u bench.py --config c2 --steps 50 --warmup 5 --no-cpu --no-extras \
    >> gpurun_out/r4t_c2.jsonl 2>> gpurun_out/r4t_c2.err
}
for rep in 1 2; do
  run default PIR_X=1 || exit $?
  run tile512 PIR_QUERY_TILE1=512 || exit $?
  run tile256 PIR_QUERY_TILE1=256 || exit $?
  run prio2 PIR_QUERY_TREE_PRIO=2 || exit $?
done
