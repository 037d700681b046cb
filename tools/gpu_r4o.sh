#!/bin/bash
# round 4, pass O: k_query's sqrt(N) mode (multiparty / covering-design shares built by the tree
# waves under the scan): its tests (forced vs two-kernel vs oracle), the cd/multiparty suites,
# and the fused-vs-two-kernel bench A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cd.py tests/test_multiparty.py tests/test_wire.py -m gpu -x -v \
  --timeout 200 --timeout-method thread > gpurun_out/r4o_pytest.log 2>&1 || exit $?
for rep in 1 2; do
  for f in 0 1; do
    for c in ccd cm ccd7; do
      echo "## fused=$f $c" >> gpurun_out/r4o_ab.jsonl
      PIR_MP_FUSED=$f timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 \
        >> gpurun_out/r4o_ab.jsonl 2>> gpurun_out/r4o_ab.err || exit $?
    done
  done
done
