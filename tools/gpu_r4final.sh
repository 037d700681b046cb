#!/bin/bash
# round 4, final: the committed tree as the driver will run it -- whole GPU suite, smoke, the
# default bench line (library e476477c, the counters' library)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
sha256sum erasurecodedpir_amd/libpir_engine.so > gpurun_out/r4final_lib_sha256.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
  > gpurun_out/r4final_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4final_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/r4final_bench.json 2> gpurun_out/r4final_bench.err
