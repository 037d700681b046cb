# round 3: kernel trace of c3b with the pipelined k_scan_t; same-box A/B with the GPR-index scan
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3i_prof -o c3b --output-format csv -- python3 bench.py --config c3b --steps 2 --warmup 1 --no-cpu --no-extras > gpurun_out/r3i_c3b_prof.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config c3b --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/r3i_c3b.log 2>&1 || exit 2
PIR_SCAN_T=0 timeout -k 10 200 python bench.py --config c3b --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/r3i_c3b_uni.log 2>&1 || exit 3
