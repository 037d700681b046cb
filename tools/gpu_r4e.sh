#!/bin/bash
# round 4, pass E: the fold's issue cost with the index written straight into M0 (micro)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 120 tools/micro/fold_issue > gpurun_out/r4e_fold_issue.txt 2>&1
