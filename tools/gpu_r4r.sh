#!/bin/bash
# round 4, pass R: rows in flight per scan lane in the four-Russians k_query (PIR_PLANE_U 8 vs
# 16, the u16 build via $PIR_ENGINE_LIB): its parity tests, then configs[4] / 3-4 rounds A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
U16=$PWD/erasurecodedpir_amd/libpir_engine_u16.so
for rep in 1 2; do
  for lib in default u16; do
    for c in c5 ccd7; do
      echo "## $lib $c" >> gpurun_out/r4r_ab.jsonl
      if [ $lib = u16 ]; then export PIR_ENGINE_LIB=$U16; else unset PIR_ENGINE_LIB; fi
      timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 --no-cpu --no-extras \
        >> gpurun_out/r4r_ab.jsonl 2>> gpurun_out/r4r_ab.err || exit $?
    done
  done
done
unset PIR_ENGINE_LIB
timeout -k 10 300 python -u tools/probe_rounds.py > gpurun_out/r4r_rounds_default.txt 2>&1 || exit $?
PIR_ENGINE_LIB=$U16 timeout -k 10 300 python -u tools/probe_rounds.py > gpurun_out/r4r_rounds_u16.txt 2>&1 || exit $?
for f in 0 1 0 1; do
  echo "## cm4 fused=$f" >> gpurun_out/r4r_cm4.jsonl
  PIR_MP_FUSED=$f timeout -k 10 300 python -u bench.py --config cm4 --steps 20 --warmup 3 --no-cpu --no-extras \
    >> gpurun_out/r4r_cm4.jsonl 2>> gpurun_out/r4r_ab.err || exit $?
done
