# round 3: k_scan_uni four-Russians coefficient words by scalar loads (PIR_M4R_SLOAD): the
# per-round diagnostic, the whole GPU suite, then a same-box A/B against the packed build
# without them (tools/_tmp_ab/libpir_engine_packed.so) on Hollanti 5 rounds (ch5)
set -o pipefail
mkdir -p gpurun_out
A=$GRAFT_REPO_ROOT/tools/_tmp_ab
timeout -k 10 120 python -u tools/diag/m4r_rounds.py > gpurun_out/r3zb_rounds.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r3zb_pytest.log 2>&1 || exit 2
for v in new old new old; do
  if [ $v = old ]; then L=$A/libpir_engine_packed.so; else L=""; fi
  PIR_ENGINE_LIB=$L timeout -k 10 200 python bench.py --config ch5 --steps 10 --warmup 3 --no-cpu --no-extras >> gpurun_out/r3zb_ch5_$v.log 2>&1 || exit 4
done
