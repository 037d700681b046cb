#!/bin/bash
# round 4, pass AF: the final library (2-share sqrt(N) k_query with 4 share waves by default):
# whole GPU suite, smoke, default bench, cm / cd2 lines, then counters at this library
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
sha256sum erasurecodedpir_amd/libpir_engine.so > gpurun_out/r4af_lib_sha256.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
  > gpurun_out/r4af_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4af_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/r4af_bench.json 2> gpurun_out/r4af_bench.err || exit $?
for c in cm ccd ccd7 cm4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 --no-cpu > gpurun_out/r4af_$c.json 2>> gpurun_out/r4af_mp.err || exit $?
done
K=10 CONFIGS="c24 c5" PASSES="traffic insts active" tools/gpu_pmc.sh > gpurun_out/r4af_pmc.txt 2>&1 || exit $?
K=10 CONFIGS="ccd cm" PASSES="traffic" tools/gpu_pmc.sh >> gpurun_out/r4af_pmc.txt 2>&1
