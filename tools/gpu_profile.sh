#!/bin/bash
# rocprofv3 passes for the committed profiles: kernel trace + stats, then separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) -- never combined with tracing domains.  W = K so every queue launch
# of the dominant kernel answers the same number of queries.  Each step time-limited.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import erasurecodedpir_amd as p; p.load()" || exit 3
K=${K:-20}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 5 "gpurun_out/$name.log"; exit $rc; fi
}
for cfg in ${CONFIGS:-c2 c24}; do
  rm -rf gpurun_out/prof_$cfg gpurun_out/pmcf_$cfg gpurun_out/pmcw_$cfg
  run trace_$cfg 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$cfg -o run --output-format csv -- python bench.py --config $cfg --steps $K --warmup $K --no-cpu --queue-only
  run pmcf_$cfg 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_$cfg -o run --output-format csv -- python bench.py --config $cfg --steps $K --warmup $K --no-cpu --queue-only
  run pmcw_$cfg 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_$cfg -o run --output-format csv -- python bench.py --config $cfg --steps $K --warmup $K --no-cpu --queue-only
done
exit 0
