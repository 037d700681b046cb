# final library (two four-Russians groups in flight): the whole -m gpu suite, then the evidence
# of tools/gpu_r7a.sh (counters, kernel traces, default command under rocprof, smoke, the default
# bench line, the explicit-share legs)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
sha256sum erasurecodedpir_amd/libpir_engine.so > gpurun_out/r7e_lib_sha256.txt &&
tools/gpu_steps.sh r7e pytest &&
CONFIGS="c24 c5" PASSES="traffic insts" bash tools/gpu_pmc.sh &&
CONFIGS="c3b" PASSES="traffic insts active lds" bash tools/gpu_pmc.sh &&
CONFIGS="ccd cm" PASSES="traffic insts" bash tools/gpu_pmc.sh &&
tools/gpu_steps.sh r7e prof:default smoke bench &&
tools/gpu_steps.sh r7f bench:--config+ch+--no-cpu+--no-extras bench:--config+ch3+--no-cpu+--no-extras bench:--config+ch5+--no-cpu+--no-extras bench:--config+ccd+--no-cpu+--no-extras bench:--config+ccd7+--no-cpu+--no-extras bench:--config+cm+--no-cpu+--no-extras bench:--config+cm4+--no-cpu+--no-extras
