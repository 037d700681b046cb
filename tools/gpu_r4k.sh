#!/bin/bash
# round 4, pass K: k_query parity on the tree-ILP default build; the multiparty /
# covering-design shares kernel at 1024 threads (16 waves per CU), tests + bench; the
# region/tile read micro; the tree-wave priority knob on lone queries
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
# the k_query parity tests on the default build (tree ILP 2 + the tile-0 row-shape last level)
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_threads.py -m gpu -x -q \
  --timeout 250 --timeout-method thread > gpurun_out/r4k_pytest.log 2>&1 || exit $?
# the multiparty / covering-design shares kernel at 1024 threads (16 waves per CU)
timeout -k 10 300 python -u -m pytest tests/test_cd.py tests/test_multiparty.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r4k_mp_pytest.log 2>&1 || exit $?
for c in ccd cm ccd7; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 \
    > gpurun_out/r4k_bench_$c.json 2>> gpurun_out/r4k_bench_mp.err || exit $?
done
timeout -k 10 300 tools/micro/read_regions > gpurun_out/r4k_read_regions.txt 2>&1
# tree-wave priority (PIR_QUERY_TREE_PRIO: s_setprio of the tree waves after the first tile) on
# the lone-query shapes, with both libraries (the default build is PIR_TREE_ILP=2 since pass J)
ILP1=$PWD/erasurecodedpir_amd/libpir_engine_ilp1.so
for rep in 1 2; do
  for lib in ilp1 ilp2; do
    for prio in 0 3; do
      if [ $lib = ilp1 ]; then export PIR_ENGINE_LIB=$ILP1; else unset PIR_ENGINE_LIB; fi
      for c in c2 c24; do
        echo "## $lib prio=$prio $c" >> gpurun_out/r4k_prio.jsonl
        PIR_QUERY_TREE_PRIO=$prio timeout -k 10 200 python -u bench.py --config $c --no-cpu --no-extras \
          --steps 10 --warmup 3 >> gpurun_out/r4k_prio.jsonl 2>> gpurun_out/r4k_prio.err || exit $?
      done
    done
  done
done
unset PIR_ENGINE_LIB
