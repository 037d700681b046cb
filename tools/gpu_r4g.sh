#!/bin/bash
# round 4, pass G: covering-design (mode 4) tests + the multiparty suite (shared evaluation path)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cd.py tests/test_multiparty.py -m gpu -x -v \
  --timeout 120 --timeout-method thread > gpurun_out/r4g_pytest.log 2>&1
