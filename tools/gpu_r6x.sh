set -o pipefail
# k_scan_uni claiming row chunks in every instance ($PIR_SCAN_DYN=1): parity, then Hollanti
# 1 / 3 / 5 rounds off against on
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
PIR_SCAN_DYN=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_m4r_folds.py tests/test_hollanti.py tests/test_multiparty.py tests/test_gpu_parity.py -k "coef or scan or holl or m4r or exchange" > gpurun_out/r6x_pytest.log 2>&1 &&
tail -2 gpurun_out/r6x_pytest.log &&
for cfg in ch ch3 ch5; do
  for i in 1 2; do
    for d in 0 1; do
      PIR_SCAN_DYN=$d timeout -k 10 240 python -u bench.py --config $cfg --no-cpu --no-extras --steps 20 --warmup 5 >> gpurun_out/r6x_coef_dyn_ab.jsonl 2>> gpurun_out/r6x_bench.err || exit 1
    done
  done
done &&
python3 -c "
import json
for ln in open('gpurun_out/r6x_coef_dyn_ab.jsonl'):
    d=json.loads(ln); print(d['config']['workload'][:60], d['ms_per_step'], d['roofline'].get('frac'))
"
