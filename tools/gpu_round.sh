#!/bin/bash
# Round-end evidence: the default bench line (CPU reference leg included), the same command under
# rocprofv3 --kernel-trace --stats (CPU leg off: its worker processes stay out of the profiler),
# and the other configs' bench lines.  Each GPU step time-limited; a failure ends the session.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 1 "gpurun_out/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
python -c "import erasurecodedpir_amd as p; p.load()" || exit 3
[ -n "$SKIP_DEFAULT" ] || step bench_default 500 python bench.py
if [ -z "$SKIP_PROF" ]; then
  rm -rf gpurun_out/prof_default
  step prof_default 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default -o run --output-format csv -- python bench.py --no-cpu
fi
for c in ${EXTRA_CONFIGS:-c5 c3 c3b ch ch3 cm cm4}; do
  step bench_$c 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu --no-extras
done
if [ -z "$SKIP_PROF" ]; then  # the coefficient-scan paths: k_mp_shares / k_interleave_coefs + k_scan_uni
  for c in cm ch3; do
    rm -rf gpurun_out/prof_$c
    step prof_$c 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- python bench.py --config $c --steps 10 --warmup 3 --no-cpu --no-extras
  done
fi
exit 0
