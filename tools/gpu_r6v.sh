# final-library evidence after the scan-evening change (sha 5e897a29; its -m gpu suite ran in
# r6u): kernel traces + PMC passes per config (tools/gpu_pmc.sh), the default bench command under
# rocprofv3 --kernel-trace --stats, smoke, and the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
sha256sum erasurecodedpir_amd/libpir_engine.so > gpurun_out/r6v_lib_sha256.txt &&
CONFIGS="c24 c5" PASSES="traffic insts" bash tools/gpu_pmc.sh &&
CONFIGS="c3b" PASSES="traffic insts active lds" bash tools/gpu_pmc.sh &&
CONFIGS="ccd cm" PASSES="traffic insts" bash tools/gpu_pmc.sh &&
tools/gpu_steps.sh r6v prof:default smoke bench
