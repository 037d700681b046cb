set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
for v in 1024 512 256 1024 512 256; do
  PIR_QUERY_TILE1=$v timeout -k 10 300 python -u bench.py --config c2 --no-cpu --no-extras --steps 20 --warmup 5 > gpurun_out/r6d_c2_t$v.json 2>> gpurun_out/r6d.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r6d_c2_t$v.json').read().strip().splitlines()[-1]); print('tile1', $v, 'lone', d['single_query']['ms_per_query'], 'queue', d['ms_per_step'])" | tee -a gpurun_out/r6d_tile1_ab.txt
done &&
for v in 1 0 1 0; do
  PIR_QUERY_SUPER=$v timeout -k 10 300 python -u bench.py --config c2 --no-cpu --no-extras --steps 20 --warmup 5 > gpurun_out/r6d_c2_s$v.json 2>> gpurun_out/r6d.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r6d_c2_s$v.json').read().strip().splitlines()[-1]); print('super', $v, 'lone', d['single_query']['ms_per_query'], 'queue', d['ms_per_step'])" | tee -a gpurun_out/r6d_tile1_ab.txt
done &&
tools/gpu_steps.sh r6d bench
