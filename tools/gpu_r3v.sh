# round 3: packed four-Russians plane indices (m4r_fold4p): the whole GPU suite, then a same-box
# A/B against the unpacked fold (tools/_tmp_ab/libpir_engine.so, -DPIR_M4R_PACKED=0) on the
# many-round shapes (configs[4] = c5 through k_query, Hollanti 5 rounds = ch5 through k_scan_uni)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r3v_pytest.log 2>&1 || exit 1
for v in new old new old; do
  if [ $v = old ]; then export PIR_ENGINE_LIB=$GRAFT_REPO_ROOT/tools/_tmp_ab/libpir_engine.so; else unset PIR_ENGINE_LIB; fi
  timeout -k 10 200 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu --no-extras >> gpurun_out/r3v_c5_$v.log 2>&1 || exit 2
  timeout -k 10 200 python bench.py --config ch5 --steps 10 --warmup 3 --no-cpu --no-extras >> gpurun_out/r3v_ch5_$v.log 2>&1 || exit 3
done
