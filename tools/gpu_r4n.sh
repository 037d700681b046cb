#!/bin/bash
# round 4, pass N: the four-Russians k_query for 3 rounds -- its parity tests (k_query m4r vs
# plane masks vs oracle, folds at full occupancy), the rounds probe, configs[4] unchanged
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_m4r_folds.py -m gpu -x -q \
  -k "m4r or fused_reduce or random_shapes" --timeout 200 --timeout-method thread > gpurun_out/r4n_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/probe_rounds.py > gpurun_out/r4n_rounds.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/probe_rounds.py >> gpurun_out/r4n_rounds.txt 2>&1
