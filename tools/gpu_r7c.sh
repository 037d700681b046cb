set -o pipefail
# Hollanti 5 rounds with 2 four-Russians groups in flight per wave (PIR_SCAN_DYN_G=2) and 3 rounds
# with 8 rows in flight (PIR_SCAN_U3=8): alt build against the default build (G=1, U3=4);
# parity of the alt build on the m4r / Hollanti tests first
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
G1=$PWD/erasurecodedpir_amd/csrc/build_alt/libpir_engine_g1.so && G2=$PWD/erasurecodedpir_amd/csrc/build_alt/libpir_engine_g2.so &&
PIR_ENGINE_LIB=$G2 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_m4r_folds.py tests/test_hollanti.py > gpurun_out/r7c_pytest.log 2>&1 &&
tail -2 gpurun_out/r7c_pytest.log &&
for cfg in ch5 ch3; do
  for i in 1 2; do
    for L in $G1 $G2; do
      PIR_ENGINE_LIB=$L timeout -k 10 240 python -u bench.py --config $cfg --no-cpu --no-extras --steps 20 --warmup 5 >> gpurun_out/r7c_ab.jsonl 2>> gpurun_out/r7c_bench.err || exit 1
      echo "$(basename $L)" >> gpurun_out/r7c_ab_libs.txt
    done
  done
done &&
python3 -c "
import json
libs=open('gpurun_out/r7c_ab_libs.txt').read().split()
for lib, ln in zip(libs, open('gpurun_out/r7c_ab.jsonl')):
    d=json.loads(ln); print(lib, d['config']['workload'][:50], d['ms_per_step'], d['roofline'].get('frac'))
"
