#!/bin/bash
# round 4, pass F: the whole GPU suite + smoke at HEAD (as the driver runs them), then the
# default bench line
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
  > gpurun_out/r4f_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/r4f_bench.json 2> gpurun_out/r4f_bench.err
