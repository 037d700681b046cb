# diagnose the packed four-Russians fold: which shapes / rounds / coefficient bits go wrong
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/diag/m4r_rounds.py > gpurun_out/r3y_rounds.log 2>&1; echo "rounds rc=$?"
exit 0
exit 0
