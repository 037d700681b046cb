set -o pipefail
# Hollanti 5 rounds: 2 / 3 / 4 four-Russians groups in flight per wave (G2 = the new default);
# parity of G3 / G4 on the fold tests
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
A=$PWD/erasurecodedpir_amd/csrc/build_alt &&
for G in 3 4; do
  PIR_ENGINE_LIB=$A/libpir_engine_g$G.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_m4r_folds.py -k scan_uni > gpurun_out/r7d_pytest_g$G.log 2>&1 && tail -1 gpurun_out/r7d_pytest_g$G.log || exit 1
done &&
for i in 1 2; do
  for G in 2 3 4; do
    PIR_ENGINE_LIB=$A/libpir_engine_g$G.so timeout -k 10 240 python -u bench.py --config ch5 --no-cpu --no-extras --steps 20 --warmup 5 >> gpurun_out/r7d_ab.jsonl 2>> gpurun_out/r7d_bench.err || exit 1
    echo "g$G" >> gpurun_out/r7d_ab_libs.txt
  done
done &&
python3 -c "
import json
libs=open('gpurun_out/r7d_ab_libs.txt').read().split()
for lib, ln in zip(libs, open('gpurun_out/r7d_ab.jsonl')):
    d=json.loads(ln); print(lib, d['config']['workload'][:50], d['ms_per_step'], d['roofline'].get('frac'))
"
