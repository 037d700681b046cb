# round 3 evidence: full GPU suite, default bench, configs[2]/Hollanti/configs[4] lines, c3b trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider --durations=10 > gpurun_out/r3g_pytest.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config c3b --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/r3g_c3b.log 2>&1 || exit 2
timeout -k 10 200 python bench.py --config ch5 --steps 5 --warmup 2 --no-cpu --no-extras > gpurun_out/r3g_ch5.log 2>&1 || exit 3
timeout -k 10 200 python bench.py --config c3 --steps 5 --warmup 2 --no-cpu --no-extras > gpurun_out/r3g_c3.log 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3g_prof -o c3b --output-format csv -- python3 bench.py --config c3b --steps 2 --warmup 1 --no-cpu --no-extras > gpurun_out/r3g_c3b_prof.log 2>&1 || exit 5
