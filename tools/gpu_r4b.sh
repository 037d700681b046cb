#!/bin/bash
# round 4, counters at HEAD: kernel trace + PMC passes (traffic, instruction mix, issue/wait
# breakdown, LDS) for the north_star shape (c24), configs[4] per server (c5) and configs[2]
# batched (c3b); the library sha is recorded beside each config's passes (tools/gpu_pmc.sh)
cd "$(dirname "$0")/.."
K=10 CONFIGS="c24 c5" PASSES="traffic insts active" tools/gpu_pmc.sh || exit $?
K=2 CONFIGS="c3b" PASSES="traffic insts active lds" tools/gpu_pmc.sh || exit $?
# the hybrid AES question: T-table and bitsliced waves on the same CU
timeout -k 10 120 tools/micro/aes_hybrid > gpurun_out/r4b_aes_hybrid.txt 2>&1 || exit $?
timeout -k 10 120 tools/micro/aes_bitsliced > gpurun_out/r4b_aes_bitsliced.txt 2>&1 || exit $?
