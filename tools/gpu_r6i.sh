set -o pipefail
# A/B of the descent CW-prefetch build against the committed build (sha 408036cb)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
OLD=$PWD/erasurecodedpir_amd/csrc/build_alt/libpir_engine_old.so &&
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --no-cpu --steps 20 --warmup 5 > gpurun_out/r6i_new_$i.json 2> gpurun_out/r6i_new_$i.err &&
  PIR_ENGINE_LIB=$OLD timeout -k 10 240 python -u bench.py --no-cpu --steps 20 --warmup 5 > gpurun_out/r6i_old_$i.json 2> gpurun_out/r6i_old_$i.err || exit 1
done &&
timeout -k 10 300 python -u tools/trace_query.py --n 20 --reps 2 > gpurun_out/r6i_trace_c2_new.log 2>&1 &&
PIR_ENGINE_LIB=$OLD timeout -k 10 300 python -u tools/trace_query.py --n 20 --reps 2 > gpurun_out/r6i_trace_c2_old.log 2>&1 &&
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r6i_*_?.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    ex=d.get('extras',{}) if isinstance(d.get('extras'),dict) else {}
    print(f, d['ms_per_step'], d['roofline']['frac'], json.dumps({k:v for k,v in d.items() if k.startswith('configs')})[:600])
PY
tail -30 gpurun_out/r6i_trace_c2_new.log; tail -30 gpurun_out/r6i_trace_c2_old.log
