# round 3: default bench line after the packed four-Russians fold, and a c5 kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/r3za_default.log 2> gpurun_out/r3za_default.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3za_prof_c5 -o c5 -- python3 bench.py --config c5 --steps 10 --warmup 3 --no-cpu --no-extras > gpurun_out/r3za_c5_prof.log 2>&1 || exit 2
