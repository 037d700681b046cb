# round 3: configs[2] batched -- kernel trace of the DFS leaf stage build, keys-per-pass sweep
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3c_prof -o c3b -- python3 bench.py --config c3b --steps 2 --warmup 1 --no-cpu --no-extras > gpurun_out/r3c_c3b_prof.log 2>&1 || exit 1
for G in 4 16; do
PIR_BENCH_BATCH_G=$G timeout -k 10 200 python bench.py --config c3b --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/r3c_c3b_g$G.log 2>&1 || exit 2
done
