"""The client-side names of package c (src/client/*.go, src/benchmark/benchmark.go bind the same
SWIG package as the server): the drop-in header set compiles and links as the revised
c.swigcxx would use it, every inventory name is in the library's dynamic symbol table, the
deterministic ones match the reference (tests/golden/client_kat.json, from libref), and the
key generators produce queries the engine answers and the client decodes."""
import ctypes
import hashlib
import hmac
import json
import os
import subprocess

import numpy as np
import pytest

import _oracle as O
from erasurecodedpir_amd import _lib

INCLUDE = os.path.join(O.ROOT, "include")
LIBDIR = os.path.dirname(_lib.LIB_PATH)


def _inventory():
    return O.golden("go_c_names.json")["names"]


def _swig_tu():
    """A C++ translation unit that uses every Go-bound name exactly as the SWIG wrapper of the
    revised c.swigcxx (INTEGRATION.md Route 1: `#include "pir_server.h"` only) does."""
    lines = ['#include "pir_server.h"', "#include <stdio.h>", "int main() {"]
    for ent in _inventory():
        c = ent["c"]
        if ent["kind"] == "function":
            lines.append(f'  printf("%p\\n", (void*)&{c});')
        elif ent["kind"] == "global":
            lines.append(f'  printf("%p\\n", (void*)&{c});')
        else:
            lines.append(f'  printf("%zu\\n", sizeof({c}));')
    lines += ["  return 0;", "}"]
    return "\n".join(lines) + "\n"


@pytest.mark.parametrize("lang", ["c++", "c"])
def test_swig_header_set_compiles_and_links(tmp_path, lang):
    """`g++ -fsyntax-only` (and gcc, for the plain-cgo Route 2) accepts exactly the header set
    of the revised c.swigcxx, and a program referencing every inventory name links against
    libpir_engine.so with no other library (no -lcrypto, no reference sources)."""
    src = tmp_path / ("tu.cpp" if lang == "c++" else "tu.c")
    src.write_text(_swig_tu())
    cc = "g++" if lang == "c++" else "gcc"
    std = "-std=c++17" if lang == "c++" else "-std=c11"
    subprocess.check_call([cc, std, "-Wall", "-Werror", "-fsyntax-only", f"-I{INCLUDE}", str(src)])
    exe = tmp_path / "tu"
    subprocess.check_call([cc, std, f"-I{INCLUDE}", str(src), "-o", str(exe), f"-L{LIBDIR}",
                           "-lpir_engine", f"-Wl,-rpath,{LIBDIR}"])
    assert exe.exists()


def test_every_inventory_name_in_dynamic_symbols():
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH], text=True)
    syms = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    missing = [(e["go"], e["c"]) for e in _inventory()
               if e["kind"] in ("function", "global") and e["c"] not in syms]
    assert not missing, missing
    assert len(_inventory()) >= 60


def test_mac_choose_keylens_match_reference():
    from erasurecodedpir_amd import server as S
    g = O.golden("client_kat.json")
    lib = _lib.load()
    for case in g["mac"]:
        key, msg = bytes.fromhex(case["key"]), bytes.fromhex(case["msg"])
        got = S.mac(key, msg)
        assert got.hex() == case["mac"]
        assert got == hmac.new(key, msg, hashlib.sha256).digest()
    for nk, v in g["choose"].items():
        n, k = map(int, nk.split(","))
        assert lib.choose(n, k) == v, nk
    for a, v in g["cd_key_len"].items():
        assert lib.calcCDDPFKeyLength(*map(int, a.split(","))) == v, a
    for a, v in g["woodruff_key_len"].items():
        assert lib.calcWoodruffKeyLength(*map(int, a.split(","))) == v, a
    r = lib.convertInt(-5)
    assert (r.lo, r.hi) == ((1 << 64) - 5, (1 << 64) - 1)  # sign-extended like (uint128_t)(int)


def test_out_of_scope_client_names_abort():
    code = ("import ctypes; from erasurecodedpir_amd import _lib; L = _lib.load(); "
            "L.generateCDQuery(None, 1, None)")
    r = subprocess.run(["python", "-c", code], cwd=O.ROOT, capture_output=True, text=True)
    assert r.returncode != 0 and "outside" in r.stderr


def _interp_coeffs(xs, ys):
    """Coefficients of the polynomial through (xs, ys) over GF(2^8)/0x11d (the oracle's
    Gauss-Jordan, coding.cpp:73-126)."""
    m = len(xs)
    V = np.array([[O.gf_pow(x, c) for c in range(m)] for x in xs], np.uint8)
    inv = np.zeros((m, m), np.uint8)
    assert O.lib().orc_gf_invert_matrix(O.P(V), O.P(inv), m) == 0
    return [np.bitwise_xor.reduce([O.gf_mul(int(inv[i, j]), int(ys[j])) for j in range(m)])
            for i in range(m)]


@pytest.mark.parametrize("L,f,t,k,r,rho", [(8, 16, 1, 2, 1, 1), (7, 30, 2, 3, 1, 1),
                                           (8, 20, 1, 4, 2, 2)])
def test_generateHollantiQuery_structure(L, f, t, k, r, rho):
    """generateHollantiQuery (genHollantiDPF, shamir_dpf.cpp:190-237): for every round a and
    record x the parties' values lie on a polynomial of t + RHO*NUM_ROUNDS coefficients whose
    coefficient t + (a+1)*RHO - 1 is [x == index] and whose other secret-block coefficients are
    0 (the t low ones random)."""
    from erasurecodedpir_amd import server as S
    S.setSystemParams(L, f, t, k, r, 0, rho, 0, 3)
    prm = S.params()
    p, nq, N = prm["NUM_PARTIES"], prm["NUM_ROUNDS"], prm["NUM_ENCODED_FILES"]
    idx = N // 3 + 1
    keys = S.generateHollantiQuery(idx)
    assert keys.shape == (p, nq, N)
    m = t + rho * nq
    assert p >= m
    xs = list(range(1, m + 1))
    for a in range(nq):
        for x in (0, idx, N - 1):
            co = _interp_coeffs(xs, keys[:m, a, x])
            for c in range(t, m):
                want = 1 if (c == t + (a + 1) * rho - 1 and x == idx) else 0
                assert co[c] == want, (a, x, c)
            if p > m:  # the extra parties lie on the same polynomial
                val = 0
                for c in reversed(range(m)):
                    val = O.gf_mul(val, m + 1) ^ int(co[c])
                assert val == keys[m, a, x]
    assert len({keys[0, 0, x] for x in range(N)}) > 8  # the low coefficients are random


@pytest.mark.gpu
def test_generate_opt_DPF_tree_query_end_to_end():
    """Keys from generate_opt_DPF_tree_query (GPU key generation) answered by every server of
    an erasure-coded setup through the shim, two servers dropped, decoded by the client
    (client.cpp:211-268) -- the src/client/tree.go flow."""
    from erasurecodedpir_amd import server as S
    L, f, k, r = 12, 16, 4, 2
    S.setSystemParams(L, f, 1, k, r, 0, 1, 0, 0)
    prm = S.params()
    p, n = prm["NUM_PARTIES"], prm["LOG_NUM_ENCODED_FILES"]
    c = S.Client(L, f)
    servers = []
    for q in range(p):
        s = S.Server(q + 1, n, f)
        c.encode_across_files_server(s)
        servers.append(s)
    for idx in (1, 7, (1 << n) - 1):
        keys = c.generate_opt_DPF_tree_query(idx)
        assert len(keys) == p and len(keys[0]) == S.calcOptimizedDPFTreeKeyLength(p, n, prm["NUM_ROUNDS"])
        ans = [servers[q].runOptimizedDPFTreeQuery(keys[q], prm["NUM_ROUNDS"]) for q in range(p)]
        er = [0 if q in (0, 3) else 1 for q in range(p)]
        dec = c.assembleDPFTreeQueryResponses(er, np.stack([ans[q] for q in range(p) if er[q]]))
        want = np.arange(f, dtype=np.uint8) if idx == 1 else np.full(f, idx & 0xFF, np.uint8)
        assert np.array_equal(dec, want), idx
    for s in servers:
        s.freeServer()
    c.free_client()


@pytest.mark.gpu
def test_generateHollantiQuery_end_to_end():
    """generateHollantiQuery keys, the engine's runHollantiQuery answers over encode-within
    shards, one server dropped, assembleHollantiResponses == the record (hollanti.go flow)."""
    from erasurecodedpir_amd import server as S
    L, f, t, k, r, rho = 10, 64, 1, 2, 1, 1
    S.setSystemParams(L, f, t, k, r, 0, rho, 0, 3)
    prm = S.params()
    p, efs = prm["NUM_PARTIES"], prm["ENCODED_FILE_SIZE_BYTES"]
    c = S.Client(L, f)
    servers = []
    for q in range(p):
        s = S.Server(q + 1, L, efs)
        c.encode_within_files_server(s)
        servers.append(s)
    for idx in (1, 300):
        keys = c.generateHollantiQuery(idx)
        ans = [servers[q].runHollantiQuery(keys[q]) for q in range(p)]
        er = [1] * p
        er[1] = 0
        dec = S.assembleHollantiResponses(er, np.stack([ans[q] for q in range(p) if er[q]]))
        want = np.arange(f, dtype=np.uint8) if idx == 1 else np.full(f, idx & 0xFF, np.uint8)
        assert np.array_equal(dec, want), idx
    for s in servers:
        s.freeServer()
    c.free_client()
