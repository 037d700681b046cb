#!/bin/bash
# round 4, pass S: kernel traces of the sqrt(N) k_query mode (ccd, ccd7, cm4), then the whole GPU
# suite + smoke + the default bench line (longer extra legs) on the final library
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for c in ccd ccd7 cm4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4s_prof_$c -o run -- \
    python3 bench.py --config $c --steps 20 --warmup 3 --no-cpu --no-extras > gpurun_out/r4s_prof_$c.log 2>&1 || exit $?
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
  > gpurun_out/r4s_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4s_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/r4s_bench.json 2> gpurun_out/r4s_bench.err
