# GPU check of the query queue: parity (stream + query subset), then queue throughput
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 tests/test_gpu_parity.py -k "stream or query or fused" > gpurun_out/pytest_q.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_q.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/stream_probe.py > gpurun_out/stream_probe.log 2>&1; rc=$?; cat gpurun_out/stream_probe.log; exit $rc
