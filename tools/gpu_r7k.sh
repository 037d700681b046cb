# final library (sqrt(N) routing by seeds a row): the whole -m gpu suite, counters, kernel traces,
# the default command under rocprof, smoke, the default bench line, the explicit-share legs
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
sha256sum erasurecodedpir_amd/libpir_engine.so > gpurun_out/r7k_lib_sha256.txt &&
tools/gpu_steps.sh r7k pytest &&
CONFIGS="c24 c5" PASSES="traffic insts" bash tools/gpu_pmc.sh &&
CONFIGS="c3b" PASSES="traffic insts active lds" bash tools/gpu_pmc.sh &&
CONFIGS="ccd cm" PASSES="traffic insts" bash tools/gpu_pmc.sh &&
tools/gpu_steps.sh r7k prof:default smoke bench &&
tools/gpu_steps.sh r7l bench:--config+ch+--no-cpu+--no-extras bench:--config+ch3+--no-cpu+--no-extras bench:--config+ch5+--no-cpu+--no-extras bench:--config+ccd+--no-cpu+--no-extras bench:--config+ccd7+--no-cpu+--no-extras bench:--config+cm+--no-cpu+--no-extras bench:--config+cm4+--no-cpu+--no-extras
