set -o pipefail
# row-chunk claiming on by default in k_scan_uni and k_scan_t: the whole -m gpu suite, then
# configs[2] (c3b) and Hollanti 5 rounds with it off / on
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
sha256sum erasurecodedpir_amd/libpir_engine.so > gpurun_out/r6y_lib_sha256.txt &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6y_pytest.log 2>&1 &&
tail -2 gpurun_out/r6y_pytest.log &&
for cfg in c3b ch5; do
  for i in 1 2; do
    for d in 0 1; do
      PIR_SCAN_DYN=$d timeout -k 10 300 python -u bench.py --config $cfg --no-cpu --no-extras --steps 5 --warmup 2 >> gpurun_out/r6y_dyn_ab.jsonl 2>> gpurun_out/r6y_bench.err || exit 1
    done
  done
done &&
python3 -c "
import json
for ln in open('gpurun_out/r6y_dyn_ab.jsonl'):
    d=json.loads(ln); print(d['config']['workload'][:60], d['ms_per_step'], d['roofline'].get('frac'))
"
