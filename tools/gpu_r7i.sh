set -o pipefail
# CD732 (4 shares, 64 seeds per row): k_query's sqrt(N) mode (PIR_MP_FUSED=1, default) against
# the separate share kernel + scan (0), and the scan priority modes in the fused one
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
for i in 1 2; do
  for m in "1 2" "0 2" "1 0"; do
    set -- $m
    PIR_MP_FUSED=$1 PIR_QUERY_SCAN_EVEN=$2 timeout -k 10 240 python -u bench.py --config ccd7 --no-cpu --no-extras >> gpurun_out/r7i_ccd7.jsonl 2>> gpurun_out/r7i.err || exit 1
    echo "fused=$1 even=$2" >> gpurun_out/r7i_modes.txt
  done
done &&
python3 -c "
import json
m=open('gpurun_out/r7i_modes.txt').read().strip().split('\n')
for k, ln in zip(m, open('gpurun_out/r7i_ccd7.jsonl')):
    d=json.loads(ln); print(k, d['ms_per_step'], d['roofline'].get('frac'))
"
