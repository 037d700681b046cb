set -o pipefail
# configs[4]: does the super-tile top stall the scan?  traces + bench with super-tiles on / off
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
timeout -k 10 300 python -u tools/trace_query.py --n 24 --p 8 --nq 5 --queue 2 --reps 1 > gpurun_out/r6j_trace_c5_super.log 2>&1 &&
PIR_QUERY_SUPER=0 timeout -k 10 300 python -u tools/trace_query.py --n 24 --p 8 --nq 5 --queue 2 --reps 1 > gpurun_out/r6j_trace_c5_nosuper.log 2>&1 &&
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --config c5 --no-cpu --no-extras --steps 20 --warmup 5 > gpurun_out/r6j_c5_super_$i.json 2> gpurun_out/r6j_c5_super_$i.err &&
  PIR_QUERY_SUPER=0 timeout -k 10 240 python -u bench.py --config c5 --no-cpu --no-extras --steps 20 --warmup 5 > gpurun_out/r6j_c5_nosuper_$i.json 2> gpurun_out/r6j_c5_nosuper_$i.err || exit 1
done &&
for f in gpurun_out/r6j_c5_*.json; do echo "$f $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['frac'])")"; done &&
grep -h "queue tile\|last_tile_ready \|end  " gpurun_out/r6j_trace_c5_*.log
