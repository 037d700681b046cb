#!/bin/bash
# round 4, pass D: the fold's issue cost (micro), lone-query knobs for configs[1]
# (12 tree + 4 scan waves; super-tiles), each against the default on the same box
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 120 tools/micro/fold_issue > gpurun_out/r4d_fold_issue.txt 2>&1 || exit $?
for v in "" "PIR_QUERY_TW=12" "PIR_QUERY_SUPER=1" "" "PIR_QUERY_TW=12" "PIR_QUERY_SUPER=1"; do
  echo "## $v" >> gpurun_out/r4d_c2_knobs.jsonl
  env $v timeout -k 10 300 python -u bench.py --config c2 --steps 20 --warmup 5 --no-cpu --no-extras \
    >> gpurun_out/r4d_c2_knobs.jsonl 2>&1 || exit $?
done
