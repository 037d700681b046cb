#!/bin/bash
# round 4, pass L: the whole GPU suite + smoke + the default bench line on the final kernels
# (tree ILP, lone-query tree priority, 16-wave shares kernel), then counters for c24 and c5 at
# this library (profiles/pmc_*.json carry its sha)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
  > gpurun_out/r4l_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4l_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/r4l_bench.json 2> gpurun_out/r4l_bench.err || exit $?
K=10 CONFIGS="c24 c5" PASSES="traffic insts active" tools/gpu_pmc.sh > gpurun_out/r4l_pmc.txt 2>&1
