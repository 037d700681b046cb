"""ctypes wrapper of oracle/liboracle.so -- the plain-C restatement of the reference path used
as the CHECKER by the tests (oracle/pir_oracle.h).  Test infrastructure only."""
import ctypes
import hashlib
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
_SO = os.path.join(ROOT, "oracle", "liboracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "oracle"])
        L = ctypes.CDLL(_SO)
        for fn in ("orc_gf_mul", "orc_gf_inv", "orc_gf_pow"):
            getattr(L, fn).restype = ctypes.c_uint8
        L.orc_blen.restype = ctypes.c_uint32
        L.orc_gen_opt_dpf.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_scan.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                               ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
        L.orc_xorshift_fill.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t]
        _lib = L
    return _lib


def P(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def u8(b):
    return np.frombuffer(bytes(b), dtype=np.uint8).copy()


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def G(seed, plen):
    out = np.zeros(plen, np.uint8)
    lib().orc_G(P(u8(seed)), plen, P(out))
    return out


def key_len(p, n, nq):
    return lib().orc_key_len(p, n, nq)


def final_cw(p, nq, rho=1):
    out = np.zeros(nq * (p - 1), np.uint8)
    lib().orc_final_cw(p, nq, rho, P(out))
    return out


def gen_keys(n, index, fcw, p, nq, seeds):
    kl = key_len(p, n, nq)
    out = np.zeros(p * kl, np.uint8)
    lib().orc_gen_opt_dpf(n, index, P(np.ascontiguousarray(fcw, np.uint8)), p, nq, P(u8(seeds)),
                          P(out))
    return [out[j * kl:(j + 1) * kl].tobytes() for j in range(p)]


def eval_all(p, party0, n, key, nq):
    out = np.zeros(nq << n, np.uint8)
    lib().orc_eval_all_opt(p, party0, n, P(u8(key)), nq, P(out))
    return out.reshape(nq, 1 << n)


def answer(p, party1, n, efs, nq, key, shard):
    out = np.zeros(nq * efs, np.uint8)
    sh = np.ascontiguousarray(shard, np.uint8)
    lib().orc_answer(p, party1, n, efs, nq, P(u8(key)), P(sh), P(out))
    return out.reshape(nq, efs)


def answer_slice(p, party1, n, efs, nq, key, shard, t, T):
    out = np.zeros(nq * efs, np.uint8)
    sh = np.ascontiguousarray(shard, np.uint8)
    lib().orc_answer_slice(p, party1, n, efs, nq, P(u8(key)), P(sh), t, T, P(out))
    return out.reshape(nq, efs)


def scan(c, shard, efs, lo=0, hi=None):
    """c: (nq, N) coefficients; shard (N*efs,) -> (nq, efs)."""
    c = np.ascontiguousarray(c, np.uint8)
    nq, N = c.shape
    n = N.bit_length() - 1
    hi = N if hi is None else hi
    out = np.zeros(nq * efs, np.uint8)
    lib().orc_scan(n, efs, nq, P(c), P(np.ascontiguousarray(shard, np.uint8)), lo, hi, P(out))
    return out.reshape(nq, efs)


def xorshift(seed, nbytes):
    out = np.zeros(nbytes, np.uint8)
    lib().orc_xorshift_fill(seed, P(out), nbytes)
    return out


def splitmix_shard(seed, row0, rows, efs):
    """The engine's fill_shard_random bytes (k_fill_shard) for rows [row0, row0 + rows)."""
    out = np.zeros(rows * efs, np.uint8)
    lib().orc_splitmix_fill(ctypes.c_uint64(seed), ctypes.c_uint64(row0), ctypes.c_uint64(rows),
                            ctypes.c_uint32(efs), P(out))
    return out


def tree_sizes(L, f, k, r, rho=1):
    s = (ctypes.c_int * 5)()
    lib().orc_tree_sizes(L, f, k, r, rho, s)
    return list(s)


def synthetic_db(L, f):
    out = np.zeros((1 << L) * f, np.uint8)
    lib().orc_synthetic_db(L, f, P(out))
    return out


def encode_across(L, f, k, p, party1, files):
    n = tree_sizes(L, f, k, 0)[1]
    out = np.zeros((1 << n) * f, np.uint8)
    lib().orc_encode_across(L, f, k, p, party1, P(np.ascontiguousarray(files, np.uint8)), P(out))
    return out


def decode(p, k, r, rho, nq, efs, erasure, responses):
    out = np.zeros(efs, np.uint8)
    lib().orc_decode(p, k, r, rho, nq, efs, P(np.asarray(erasure, np.uint8)),
                     P(np.ascontiguousarray(responses, np.uint8)), P(out))
    return out


def gf_mul(a, b):
    return lib().orc_gf_mul(a, b)


def gf_pow(a, e):
    return lib().orc_gf_pow(a, e)


# ---- multiparty sqrt(N) DPF (mode 1) ---------------------------------------------------------
def mp_sizes(p, n, t):
    """{nrk, p2, mu, nu, eval_bytes, key_len} (multiparty_dpf.cpp:470-478, utils.cpp:105-116)."""
    o = (ctypes.c_uint64 * 6)()
    lib().orc_mp_sizes(p, n, t, o)
    return dict(zip(("nrk", "p2", "mu", "nu", "eval_bytes", "key_len"), [int(v) for v in o]))


def mp_key(p, n, t, seed):
    """A synthetic multiparty key: xorshift bytes over max(eval_bytes, key_len), with the toggle
    bytes mapped to {0, 1, the raw byte} (raw % 3), so toggles are both set and clear.  The
    evaluation is a function of the key bytes: the reference's own key generation cannot make
    a usable key (RSS_SUBSETS is never filled, params.cpp:613-617)."""
    z = mp_sizes(p, n, t)
    key = xorshift(seed, max(z["eval_bytes"], z["key_len"], 16))
    lo = z["nu"] * 16 * z["p2"]
    hi = lo + z["nrk"] * z["nu"] * z["p2"]
    tb = key[lo:hi]
    key[lo:hi] = np.where(tb % 3 == 0, 0, np.where(tb % 3 == 1, 1, tb))
    return key


def mp_eval(p, n, t, key, thread_num=0, num_threads=1):
    z = mp_sizes(p, n, t)
    out = np.zeros(z["nrk"] << n, np.uint8)
    lib().orc_mp_eval(p, n, t, P(np.ascontiguousarray(key, np.uint8)), thread_num, num_threads,
                      P(out))
    return out.reshape(z["nrk"], 1 << n)


def mp_answer(p, t, n, efs, key, shard, thread_num=0, num_threads=1):
    z = mp_sizes(p, n, t)
    out = np.zeros(z["nrk"] * efs, np.uint8)
    lib().orc_mp_answer(p, t, n, efs, P(np.ascontiguousarray(key, np.uint8)),
                        P(np.ascontiguousarray(shard, np.uint8)), thread_num, num_threads, P(out))
    return out.reshape(z["nrk"], efs)


# ---- covering-design sqrt(N) DPF (mode 4) ----------------------------------------------------
def cd_sizes(n, q_needed, num_cd_keys):
    """{nrk, p2, mu, nu, eval_bytes, key_len} of evalAllCDThread (multiparty_dpf.cpp:620-625,
    utils.cpp:118-129): p2 = 2^(q_needed-1), mu = 2^(n//2+3), nrk = NUM_CD_KEYS."""
    o = (ctypes.c_uint64 * 6)()
    lib().orc_cd_sizes(n, q_needed, num_cd_keys, o)
    return dict(zip(("nrk", "p2", "mu", "nu", "eval_bytes", "key_len"), [int(v) for v in o]))


def cd_key(n, q_needed, num_cd_keys, seed):
    """A synthetic covering-design key (the evaluation is a function of the key bytes; the
    fixtures of tests/golden/cd.json hold the reference's own genCDDPF keys): xorshift bytes,
    toggle bytes mapped to {0, 1, the raw byte} as mp_key."""
    z = cd_sizes(n, q_needed, num_cd_keys)
    key = xorshift(seed, max(z["eval_bytes"], 16))
    lo = z["nu"] * 16 * z["p2"]
    hi = lo + z["nrk"] * z["nu"] * z["p2"]
    tb = key[lo:hi]
    key[lo:hi] = np.where(tb % 3 == 0, 0, np.where(tb % 3 == 1, 1, tb))
    return key


def cd_eval(n, q_needed, num_cd_keys, key, thread_num=0, num_threads=1):
    z = cd_sizes(n, q_needed, num_cd_keys)
    out = np.zeros(z["nrk"] << n, np.uint8)
    lib().orc_cd_eval(n, q_needed, num_cd_keys, P(np.ascontiguousarray(key, np.uint8)),
                      thread_num, num_threads, P(out))
    return out.reshape(z["nrk"], 1 << n)


def cd_answer(n, q_needed, num_cd_keys, efs, key, shard, thread_num=0, num_threads=1):
    """runCDQueryThread (server.cpp:443-492) on one thread's slice of rows."""
    z = cd_sizes(n, q_needed, num_cd_keys)
    out = np.zeros(z["nrk"] * efs, np.uint8)
    lib().orc_cd_answer(n, q_needed, num_cd_keys, efs, P(np.ascontiguousarray(key, np.uint8)),
                        P(np.ascontiguousarray(shard, np.uint8)), thread_num, num_threads, P(out))
    return out.reshape(z["nrk"], efs)
