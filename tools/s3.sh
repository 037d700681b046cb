cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
SKIP_PROF=1 SKIP_C24=1 bash tools/gpu_session.sh || exit $?
CONFIGS="c2 c24" bash tools/gpu_profile.sh || exit $?
