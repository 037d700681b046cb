set -o pipefail
# configs[4]: tree phases of a tile while the tree is ahead (tile 4) and behind (tile 12)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
ALT=$PWD/erasurecodedpir_amd/csrc/build_alt/libpir_engine_tt.so &&
PIR_ENGINE_LIB=$ALT PIR_TRACE_TILES=4,12 timeout -k 10 300 python -u tools/trace_query.py --n 24 --p 8 --nq 5 --queue 2 --reps 2 > gpurun_out/r6m_trace_c5_tiles_4_12.log 2>&1 &&
PIR_ENGINE_LIB=$ALT PIR_TRACE_TILES=5,13 timeout -k 10 300 python -u tools/trace_query.py --n 24 --p 8 --nq 5 --queue 2 --reps 1 > gpurun_out/r6m_trace_c5_tiles_5_13.log 2>&1 &&
PIR_ENGINE_LIB=$ALT PIR_TRACE_TILES=9,10 timeout -k 10 300 python -u tools/trace_query.py --n 24 --p 8 --nq 5 --queue 2 --reps 1 > gpurun_out/r6m_trace_c5_tiles_9_10.log 2>&1 &&
PIR_TRACE_NOSCAN=1 PIR_ENGINE_LIB=$ALT PIR_TRACE_TILES=4,12 timeout -k 10 300 python -u tools/trace_query.py --n 24 --p 8 --nq 5 --queue 2 --reps 1 > gpurun_out/r6m_trace_c5_tiles_noscan.log 2>&1 &&
grep -h "tree tile\|queue tile" gpurun_out/r6m_trace_c5_*.log
