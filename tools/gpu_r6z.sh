set -o pipefail
# Hollanti 3 rounds through the four-Russians k_scan_uni ($PIR_SCAN_M4R3=1, the new default)
# against the plane-mask fold (0): parity, then A/B
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_m4r_folds.py tests/test_hollanti.py > gpurun_out/r6z_pytest.log 2>&1 &&
tail -2 gpurun_out/r6z_pytest.log &&
for i in 1 2; do
  for d in 0 1; do
    PIR_SCAN_M4R3=$d timeout -k 10 240 python -u bench.py --config ch3 --no-cpu --no-extras --steps 20 --warmup 5 >> gpurun_out/r6z_ch3_ab.jsonl 2>> gpurun_out/r6z_bench.err || exit 1
  done
done &&
python3 -c "
import json
for ln in open('gpurun_out/r6z_ch3_ab.jsonl'):
    d=json.loads(ln); print(d['config']['workload'][:60], d['ms_per_step'], d['roofline'].get('frac'))
"
