set -o pipefail
# configs[4]: per-scan-wave consumed stamps -- does the scan waves' spread block the tree's ring?
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
ALT=$PWD/erasurecodedpir_amd/csrc/build_alt/libpir_engine_tt.so &&
PIR_ENGINE_LIB=$ALT PIR_TRACE_TILES=4,12 timeout -k 10 300 python -u tools/trace_query.py --n 24 --p 8 --nq 5 --queue 2 --reps 1 > gpurun_out/r6n_trace_c5_4_12.log 2>&1 &&
PIR_ENGINE_LIB=$ALT PIR_TRACE_TILES=8,30 timeout -k 10 300 python -u tools/trace_query.py --n 24 --p 8 --nq 5 --queue 2 --reps 1 > gpurun_out/r6n_trace_c5_8_30.log 2>&1 &&
grep -h -A1 "tree tile" gpurun_out/r6n_trace_c5_*.log
