#!/bin/bash
# GPU session: the -m gpu suite, smoke, the default bench (c24 + extras + CPU reference leg) and
# optional extra bench configs.  Every GPU step has its own time limit; a crash, abort or
# timeout ends the session (nothing further runs on the GPU).
#   SKIP_TESTS=1  TESTS="tests/x.py ..."  SKIP_BENCH=1  EXTRA_CONFIGS="c5 c3b"  BENCH_ARGS=...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
python -c "import erasurecodedpir_amd as p; p.load()" || { echo "library does not load"; exit 3; }
if [ -z "$SKIP_TESTS" ]; then
  step pytest_gpu 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 150 --timeout-method thread
  step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
fi
[ -n "$SKIP_BENCH" ] || step bench 500 python bench.py --steps 20 --warmup 5 $BENCH_ARGS
for c in $EXTRA_CONFIGS; do step bench_$c 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu --no-extras; done
exit 0
