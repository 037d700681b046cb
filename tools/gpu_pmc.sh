#!/bin/bash
# rocprofv3 passes for profiles/: kernel trace + stats per config, then PMC passes (each its own
# run, --pmc never combined with tracing domains, each under `timeout -s KILL 60`).  W = K so
# every launch of the query kernel answers the same number of queries.
#   CONFIGS="c24 c5"  K=20  PASSES="traffic insts"  LIST=1 (rocprofv3 -L into gpurun_out/)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import erasurecodedpir_amd as p; p.load()" || exit 3
K=${K:-20}
fatal() { [ "$1" = 124 ] || [ "$1" = 137 ] || [ "$1" = 134 ] || [ "$1" = 139 ]; }
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -s KILL "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 5 "gpurun_out/$name.log"; fi
  if fatal $rc; then echo "stopping after $name"; exit $rc; fi
  return 0
}
if [ -n "$LIST" ]; then
  run list 60 rocprofv3 -L
fi
BENCH="python bench.py --steps $K --warmup $K --no-cpu --queue-only"
for cfg in ${CONFIGS:-c24}; do
  rm -rf gpurun_out/prof_$cfg
  # the library these counters describe (bench.py flags a summary whose sha differs as stale)
  sha256sum erasurecodedpir_amd/libpir_engine.so > gpurun_out/pmc_${cfg}_lib_sha256.txt
  run trace_$cfg 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$cfg -o run --output-format csv -- $BENCH --config $cfg
  for pass in ${PASSES:-traffic insts}; do
    case $pass in
      traffic) sets="FETCH_SIZE WRITE_SIZE" ;;
      insts) sets="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,GRBM_GUI_ACTIVE,GRBM_COUNT" ;;
      active) sets="SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_MISC,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY,SQ_INST_CYCLES_SALU" ;;
      lds) sets="SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_LDS,GRBM_GUI_ACTIVE" ;;
      *) sets=$pass ;;
    esac
    for s in $sets; do
      tag=$(echo "$s" | tr ',' '\n' | head -n 1 | tr 'A-Z' 'a-z')
      rm -rf gpurun_out/pmc_${cfg}_$tag
      run pmc_${cfg}_$tag 60 rocprofv3 --pmc $(echo "$s" | tr ',' ' ') -d gpurun_out/pmc_${cfg}_$tag -o run --output-format csv -- $BENCH --config $cfg
    done
  done
done
exit 0
