"""The pir_server.h shim's concurrency under ThreadSanitizer, on the CPU (SURVEY.md section 5:
"Build tests under ASan/TSan on the CPU backend").  tests/tsan/ builds the shim
(erasurecodedpir_amd/csrc/pir_server.cpp, unchanged) with -fsanitize=thread against an
oracle-backed stub of the engine's device side and runs the scenarios of tests/tsan/
shim_threads.cpp: T = 16 concurrent runOptimizedDPFTreeQueryThread calls, interleaved queries,
a shard change (pirServerSetRows + pirServerShardChanged) during a slice group, 12 queries at
once (more slice groups than the shim keeps), two pirRunTreeQueryThreads fan-outs, and a GPU-path
setup with pirServerSyncRows racing the queries.  Clean = no TSan report and every answer equal
to the oracle's.  (The round-4 shim, built the same way, reports the data race on `dirty` in
pirServerShardChanged that this round fixed: profiles/r05/tsan_round4_shim.txt.)"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TSAN = os.path.join(ROOT, "tests", "tsan")


def _have_tsan(tmp_path):
    src = tmp_path / "t.cpp"
    src.write_text("int main() { return 0; }\n")
    r = subprocess.run(["g++", "-fsanitize=thread", str(src), "-o", str(tmp_path / "t")],
                       capture_output=True)
    return r.returncode == 0


def test_shim_threads_clean_under_tsan(tmp_path):
    if not shutil.which("g++") or not _have_tsan(tmp_path):
        pytest.skip("no g++ with ThreadSanitizer here")
    subprocess.check_call(["make", "-s", "-C", TSAN], stdout=subprocess.DEVNULL)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66 second_deadlock_stack=1",
               PIR_SLICE_JOIN_US="20000")  # fan-outs meet in one group under TSan's slow thread starts
    r = subprocess.run([os.path.join(TSAN, "build", "shim_threads")], capture_output=True,
                       text=True, env=env, timeout=600)
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, (r.stdout, r.stderr[-4000:])
    assert "ok: 0 failure(s)" in r.stdout
