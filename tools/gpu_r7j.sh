set -o pipefail
# the other sqrt(N) shapes (CD842, multiparty 2 / 3 shares): fused (k_query sqrt(N) mode) against
# the separate share kernel + scan
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
for cfg in ccd cm cm4; do
  for i in 1 2; do
    for f in 1 0; do
      PIR_MP_FUSED=$f timeout -k 10 240 python -u bench.py --config $cfg --no-cpu --no-extras >> gpurun_out/r7j_mp.jsonl 2>> gpurun_out/r7j.err || exit 1
      echo "$cfg fused=$f" >> gpurun_out/r7j_modes.txt
    done
  done
done &&
python3 -c "
import json
m=open('gpurun_out/r7j_modes.txt').read().strip().split('\n')
for k, ln in zip(m, open('gpurun_out/r7j_mp.jsonl')):
    d=json.loads(ln); print(k, d['ms_per_step'], d['roofline'].get('frac'))
"
