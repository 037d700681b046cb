#!/bin/bash
# One parametrised GPU-box run (replaces the one-shot tools/gpu_r*.sh lease scripts of rounds
# 3-4): a list of steps, each under its own time limit, stopping at the first failure.  Output
# goes to gpurun_out/<tag>_*; copy what is worth keeping into profiles/<round>/.
#
#   tools/gpu_steps.sh TAG STEP [STEP ...]      (run on the box: gpurun -- tools/gpu_steps.sh ...)
#
# steps:
#   env:K=V[,K=V...]      export variables for the steps after it (env: alone clears nothing)
#   pytest[:ARGS]         python -m pytest -m gpu ARGS (default: tests) -> TAG_pytest.log
#   smoke                 __graft_entry__.smoke()                        -> TAG_smoke.log
#   bench[:ARGS]          python bench.py ARGS (spaces as '+')            -> TAG_bench.jsonl
#   prof:NAME[:ARGS]      rocprofv3 --kernel-trace --stats of bench.py ARGS -> TAG_prof_NAME/
#   py:SCRIPT[:ARGS]      python tools/SCRIPT ARGS                         -> TAG_SCRIPT.log
#   sha                   sha256 of the libraries                          -> TAG_lib_sha256.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
tag=$1
shift
mkdir -p gpurun_out
out=gpurun_out/$tag
plus() { echo "${1//+/ }"; }
for step in "$@"; do
  kind=${step%%:*}
  rest=${step#*:}
  [ "$rest" = "$step" ] && rest=""
  echo "[gpu_steps] $(date +%T) $step"
  case $kind in
    env)
      IFS=',' read -ra kv <<< "$rest"
      for x in "${kv[@]}"; do export "$x"; done
      ;;
    pytest)
      args=$(plus "${rest:-tests}")
      # shellcheck disable=SC2086
      timeout -k 10 900 python -u -m pytest $args -m gpu -x -v --timeout 120 \
        --timeout-method thread > "${out}_pytest.log" 2>&1 || { tail -30 "${out}_pytest.log"; exit 1; }
      tail -3 "${out}_pytest.log"
      ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "${out}_smoke.log" 2>&1 \
        || { tail -20 "${out}_smoke.log"; exit 1; }
      tail -1 "${out}_smoke.log"
      ;;
    bench)
      # shellcheck disable=SC2086
      timeout -k 10 600 python -u bench.py $(plus "$rest") >> "${out}_bench.jsonl" 2>> "${out}_bench.err" \
        || { tail -20 "${out}_bench.err"; exit 1; }
      tail -c 400 "${out}_bench.jsonl"; echo
      ;;
    prof)
      name=${rest%%:*}
      args=${rest#*:}
      [ "$args" = "$rest" ] && args=""
      # shellcheck disable=SC2086
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "${out}_prof_${name}" -o run --output-format csv \
        -- python3 -u bench.py $(plus "$args") > "${out}_prof_${name}.log" 2>&1 \
        || { tail -20 "${out}_prof_${name}.log"; exit 1; }
      ;;
    py)
      script=${rest%%:*}
      args=${rest#*:}
      [ "$args" = "$rest" ] && args=""
      # shellcheck disable=SC2086
      timeout -k 10 600 python -u "tools/$script" $(plus "$args") >> "${out}_${script%.py}.log" 2>&1 \
        || { tail -20 "${out}_${script%.py}.log"; exit 1; }
      tail -25 "${out}_${script%.py}.log"
      ;;
    sha)
      sha256sum erasurecodedpir_amd/*.so > "${out}_lib_sha256.txt"
      ;;
    *)
      echo "unknown step $step"; exit 2
      ;;
  esac
done
echo "[gpu_steps] $(date +%T) done"
