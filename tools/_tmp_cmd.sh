set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_default.log | cut -c 1-250
rm -rf gpurun_out/prof_c2def
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2def -o run --output-format csv -- python bench.py --no-cpu > gpurun_out/prof_c2def.log 2>&1 || exit $?
grep -h '^{' gpurun_out/prof_c2def.log | cut -c 1-200
