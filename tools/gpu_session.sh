#!/bin/bash
# GPU session: gpu tests, bench (c2 with CPU baseline, c24), rocprofv3 kernel trace of c2.
# Every GPU step has its own time limit; a crash/timeout stops the session.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return $rc
}
python -c "import erasurecodedpir_amd as p; p.load()" || { echo "library does not load"; exit 3; }
[ -n "$SKIP_TESTS" ] || step pytest_gpu 900 python -m pytest tests -m gpu -x -q
step bench_c2 300 python bench.py --steps 50 --warmup 5
[ -n "$SKIP_C24" ] || step bench_c24 300 python bench.py --config c24 --steps 20 --warmup 3 --no-cpu
for c in $EXTRA_CONFIGS; do step bench_$c 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu; done
if [ -z "$SKIP_PROF" ]; then
  rm -rf gpurun_out/prof_c2
  step rocprof_c2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu
fi
exit 0
