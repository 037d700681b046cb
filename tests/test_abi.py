"""The C-ABI library: loads without a GPU, exports every function include/*.h declares, and its
pure-host pieces (sizing globals, key lengths, finalCW) agree with the reference fixtures.
No GPU compute is called here."""
import os
import re

import numpy as np
import pytest

import _oracle as O
from erasurecodedpir_amd import _lib

INCLUDE = os.path.join(O.ROOT, "include")


def declared_functions():
    names = set()
    for h in sorted(os.listdir(INCLUDE)):
        if not h.endswith(".h"):
            continue
        src = open(os.path.join(INCLUDE, h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"//[^\n]*", "", src)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b([A-Za-z_]\w*)\s*\([^;{]*\)\s*;", src, re.M):
            if not m.group(0).lstrip().startswith(("typedef", "#", "return")):
                names.add(m.group(1))
    return names


def test_library_loads_and_exports_every_declared_symbol():
    lib = _lib.load()
    names = declared_functions()
    assert {"pir_engine_create", "pir_engine_answer", "runOptimizedDPFTreeQuery",
            "runOptimizedDPFTreeQueryThread", "assemblDPFTreeQueryThreadResults",
            "pir_gen_keys"} <= names
    missing = [n for n in sorted(names) if not hasattr(lib, n)]
    assert not missing, missing
    # and the ctypes prototypes cover exactly the declared surface
    assert names == set(_lib.PROTOTYPES)


def declared_globals_and_types():
    src = "".join(open(os.path.join(INCLUDE, h)).read() for h in sorted(os.listdir(INCLUDE))
                  if h.endswith(".h"))
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    glob = set(re.findall(r"^extern\s+[\w\s\*]+?\b([A-Za-z_]\w*)\s*;", src, re.M))
    types = set(re.findall(r"}\s*([A-Za-z_]\w*)\s*;", src))
    return glob, types


def test_header_declares_every_go_bound_name():
    """Every name the reference's Go server side binds from package c (src/server/*.go,
    src/server_util/*.go; inventory tests/golden/go_c_names.json from tools/go_c_names.py) is
    declared by include/pir_server.h and exported by the library: SWIG over the drop-in header
    generates the same Go names, so package server_util compiles against it unchanged."""
    inv = O.golden("go_c_names.json")["names"]
    funcs = declared_functions()
    glob, types = declared_globals_and_types()
    lib = _lib.load()
    missing = []
    for ent in inv:
        kind, c = ent["kind"], ent["c"]
        if kind == "function":
            ok = c in funcs and hasattr(lib, c)
        elif kind == "global":
            ok = c in glob and hasattr(lib, c)
        else:  # a struct type, its SWIG constructor / destructor
            ok = c in types
        if not ok:
            missing.append((ent["go"], c, ent["sites"][0]))
    assert len(inv) >= 30
    assert not missing, missing


def test_out_of_scope_modes_refuse_loudly():
    """Modes the engine does not serve abort with a message (like the reference's
    handleErrors), in a child process."""
    import subprocess
    import sys
    code = ("from erasurecodedpir_amd import server as S; "
            "S.setSystemParams(10, 64, 2, 2, 0, 0, 1, 0, 2)")
    r = subprocess.run([sys.executable, "-c", code], cwd=O.ROOT, capture_output=True, text=True)
    assert r.returncode != 0 and "outside the engine's scope" in r.stderr


def test_hollanti_sizing_matches_reference():
    from erasurecodedpir_amd import server
    for case in O.golden("hollanti.json")["cases"]:
        server.setSystemParams(case["L"], case["f"], case["t"], case["k"], case["r"], 0,
                               case["rho"], 0, 3)
        prm = server.params()
        assert (prm["NUM_PARTIES"], prm["ENCODED_FILE_SIZE_BYTES"], prm["NUM_ROUNDS"],
                prm["NUM_ENCODED_FILES"], prm["ENCODE_ACROSS"]) == \
            (case["p"], case["efs"], case["nq"], 1 << case["L"], 0)


def test_shamir_lengths_match_reference():
    from erasurecodedpir_amd import _lib as L
    lib = L.load()
    for n, want in O.golden("hollanti.json")["shamir_key_len"].items():
        assert lib.calcShamirDPFKeyLength(int(n)) == want
        assert lib.calcShamirResponseLength(int(n), 100) == (want + 2) * 100


def test_globals_exported():
    for g in _lib.GLOBALS_INT + _lib.GLOBALS_U32:
        _lib.global_int(g)


def test_key_len_matches_reference():
    g = O.golden("prg_kat.json")
    from erasurecodedpir_amd import key_len
    from erasurecodedpir_amd.server import calcOptimizedDPFTreeKeyLength
    for k, kl in g["key_len"].items():
        p, n, nq = map(int, k.split(","))
        assert key_len(p, n, nq) == kl
        assert calcOptimizedDPFTreeKeyLength(p, n, nq) == kl


@pytest.mark.parametrize("ci", range(5))
def test_setSystemParams_sizing_matches_reference(ci):
    from erasurecodedpir_amd import server
    case = O.golden("e2e.json")["cases"][ci]
    server.setSystemParams(case["L"], case["f"], 1, case["k"], case["r"], 0, case["rho"], 0, 0)
    prm = server.params()
    assert prm["NUM_PARTIES"] == case["p"]
    assert prm["LOG_NUM_ENCODED_FILES"] == case["n"]
    assert prm["ENCODED_FILE_SIZE_BYTES"] == case["efs"]
    assert prm["NUM_ROUNDS"] == case["nq"]
    assert prm["NUM_ENCODED_FILES"] == 1 << case["n"]
    assert prm["NUM_RESPONSES"] == case["p"] - case["r"]


def test_final_cw_matches_reference():
    from erasurecodedpir_amd.client import final_cw
    for case in O.golden("dpf_eval.json")["cases"]:
        p, nq = case["p"], case["nq"]
        assert final_cw(p, nq, 1).tobytes().hex() == case["final_cw"]
    for p, nq, rho in [(8, 5, 1), (17, 16, 1), (6, 2, 2), (9, 3, 3)]:
        assert np.array_equal(final_cw(p, nq, rho), O.final_cw(p, nq, rho))


def test_errors_are_loud_without_a_gpu():
    """On a host without a usable device the engine refuses (no silent CPU path)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from erasurecodedpir_amd import Engine, PirError
    with pytest.raises(PirError):
        Engine(2, 1, 10, 16, 1)


def test_cd_key_counts_reset_per_setup():
    """setSystemParams starts from a fresh process's covering-design counts (params.cpp:368-369,
    NUM_CD_KEYS = 2, NUM_CD_KEYS_NEEDED = 4): a CD842 setup (K = 2, B = 1: p = 8, M = 2 ->
    3 / 6, params.cpp:519-599) followed by a mode-4 setup that matches no covering design
    (T = 2, K = 1, R = 1, B = 0: p = 8, M = 4) leaves the CD532 defaults, not CD842's counts."""
    from erasurecodedpir_amd import _lib as L
    from erasurecodedpir_amd import server
    server.setSystemParams(10, 64, 2, 2, 0, 1, 1, 0, 4)
    assert (L.global_int("NUM_PARTIES"), L.global_int("NUM_CD_KEYS"),
            L.global_int("NUM_CD_KEYS_NEEDED")) == (8, 3, 6)
    server.setSystemParams(10, 64, 2, 1, 1, 0, 1, 0, 4)
    assert (L.global_int("NUM_PARTIES"), L.global_int("NUM_CD_KEYS"),
            L.global_int("NUM_CD_KEYS_NEEDED")) == (8, 2, 4)
