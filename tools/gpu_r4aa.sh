#!/bin/bash
set -o pipefail
cd /root/repo
for rep in 1 2; do
  for t in 4096 1024; do
    echo "## tileq=$t" >> gpurun_out/r4aa.jsonl
    PIR_QUERY_TILEQ=$t timeout -k 10 300 python -u bench.py --config c24 --steps 20 --warmup 5 --no-cpu --no-extras --queue-only >> gpurun_out/r4aa.jsonl 2>> gpurun_out/r4aa.err || exit $?
  done
done
