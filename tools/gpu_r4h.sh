#!/bin/bash
# round 4, pass H: the wire tests (CD732_SEARCH loopback against the reference's answers), the
# covering-design bench configs, and their kernel stats
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_wire.py -m gpu -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/r4h_wire.log 2>&1 || exit $?
for c in ccd ccd7 cm; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 \
    > gpurun_out/r4h_bench_$c.json 2> gpurun_out/r4h_bench_$c.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4h_prof_ccd -o run -- \
  python3 bench.py --config ccd --steps 20 --warmup 3 > gpurun_out/r4h_prof_ccd.log 2>&1
