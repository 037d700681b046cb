# final-library evidence after the chunk-claiming scans (sha 484eb0f3; its -m gpu suite ran in
# r6y): kernel traces + PMC passes per config, the default command under rocprofv3, smoke, the
# default bench line, then the explicit-share legs (Hollanti 1/3/5, CD842/CD732, multiparty)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
sha256sum erasurecodedpir_amd/libpir_engine.so > gpurun_out/r7a_lib_sha256.txt &&
CONFIGS="c24 c5" PASSES="traffic insts" bash tools/gpu_pmc.sh &&
CONFIGS="c3b" PASSES="traffic insts active lds" bash tools/gpu_pmc.sh &&
CONFIGS="ccd cm" PASSES="traffic insts" bash tools/gpu_pmc.sh &&
tools/gpu_steps.sh r7a prof:default smoke bench &&
tools/gpu_steps.sh r7b bench:--config+ch+--no-cpu+--no-extras bench:--config+ch3+--no-cpu+--no-extras bench:--config+ch5+--no-cpu+--no-extras bench:--config+ccd+--no-cpu+--no-extras bench:--config+ccd7+--no-cpu+--no-extras bench:--config+cm+--no-cpu+--no-extras bench:--config+cm4+--no-cpu+--no-extras
