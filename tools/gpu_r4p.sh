#!/bin/bash
# round 4, pass P: the 2-share multiparty answer (cm) in k_query's sqrt(N) mode -- tile and
# tree-wave variants against the two-kernel path
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() {  # label, env...
  echo "## $*" >> gpurun_out/r4p_ab.jsonl
  env "${@:2}" timeout -k 10 300 python -u bench.py --config cm --steps 20 --warmup 3 \
    >> gpurun_out/r4p_ab.jsonl 2>> gpurun_out/r4p_ab.err
}
for rep in 1 2; do
  run two PIR_MP_FUSED=0 || exit $?
  run fused PIR_MP_FUSED=2 || exit $?
  run fused_t4096 PIR_MP_FUSED=2 PIR_QUERY_TILE1=4096 || exit $?
  run fused_prio0 PIR_MP_FUSED=2 PIR_QUERY_TREE_PRIO=0 || exit $?
done
