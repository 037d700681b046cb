set -o pipefail
# k_scan_uni four-Russians waves claiming row chunks ($PIR_SCAN_DYN=1) against fixed ranges:
# parity (m4r fold tests, Hollanti tests) with it on, then Hollanti 5 rounds A/B
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
PIR_SCAN_DYN=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_m4r_folds.py tests/test_hollanti.py > gpurun_out/r6w_pytest.log 2>&1 &&
tail -2 gpurun_out/r6w_pytest.log &&
for i in 1 2; do
  for d in 0 1; do
    PIR_SCAN_DYN=$d timeout -k 10 240 python -u bench.py --config ch5 --no-cpu --no-extras --steps 20 --warmup 5 >> gpurun_out/r6w_ch5_dyn_ab.jsonl 2>> gpurun_out/r6w_bench.err || exit 1
  done
done &&
python3 -c "
import json
for ln in open('gpurun_out/r6w_ch5_dyn_ab.jsonl'):
    d=json.loads(ln); print(d['ms_per_step'], d['roofline'].get('frac'))
"
