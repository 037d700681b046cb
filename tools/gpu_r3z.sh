# round 3: packed four-Russians indices with the readlane wait state (tools/gen_m4r.py): the
# per-round diagnostic, the whole GPU suite, then a same-box A/B against the unpacked fold
# (tools/_tmp_ab/libpir_engine.so, -DPIR_M4R_PACKED=0) on configs[4] (c5) and Hollanti 5 rounds (ch5)
set -o pipefail
mkdir -p gpurun_out
A=$GRAFT_REPO_ROOT/tools/_tmp_ab
timeout -k 10 120 python -u tools/diag/m4r_rounds.py > gpurun_out/r3z_rounds.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r3z_pytest.log 2>&1 || exit 2
for v in new old new old; do
  if [ $v = old ]; then L=$A/libpir_engine.so; else L=""; fi
  PIR_ENGINE_LIB=$L timeout -k 10 200 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu --no-extras >> gpurun_out/r3z_c5_$v.log 2>&1 || exit 3
  PIR_ENGINE_LIB=$L timeout -k 10 200 python bench.py --config ch5 --steps 10 --warmup 3 --no-cpu --no-extras >> gpurun_out/r3z_ch5_$v.log 2>&1 || exit 4
done
