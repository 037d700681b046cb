# round 3: default bench line (with the configs[2]/configs[4] legs) + c3b PMC passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/r3k_default.log 2> gpurun_out/r3k_default.err || exit 1
echo "default bench done at ${SECONDS}s" >> gpurun_out/r3k_default.err
CONFIGS=c3b K=2 PASSES="insts lds traffic" bash tools/gpu_pmc.sh > gpurun_out/r3k_pmc.log 2>&1 || exit 2
