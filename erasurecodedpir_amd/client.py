"""Client-side helpers (include/pir_client.h): DPF key generation on the GPU and the finalCW
values of generate_opt_DPF_tree_query (src/c/client.cpp:144-153)."""
import ctypes
import os

import numpy as np

from . import _lib
from ._lib import check
from .engine import key_len


def final_cw(p, nq, rho=1):
    """nq*(p-1) bytes: out[a*(p-1) + j-2] = gf_pow(j, rho*(a+1)) ^ 1, j = 2..p."""
    out = np.zeros(nq * (p - 1), np.uint8)
    _lib.load().pir_final_cw(p, nq, rho, out.ctypes.data_as(ctypes.c_void_p))
    return out


def gen_keys(n, index, p, nq=1, fcw=None, rho=1, seeds=None, device=0):
    """genOptimizedDPF (src/c/dpf_tree.cpp:142-274) on the GPU.  Returns p keys (bytes).

    seeds: p*16 root-seed bytes (the reference draws them from RAND_bytes); default
    os.urandom."""
    if fcw is None:
        fcw = final_cw(p, nq, rho)
    fcw = np.ascontiguousarray(fcw, dtype=np.uint8)
    if seeds is None:
        seeds = os.urandom(16 * p)
    seeds = np.frombuffer(bytes(seeds), dtype=np.uint8).copy()
    kl = key_len(p, n, nq)
    out = np.zeros(p * kl, np.uint8)
    check(_lib.load().pir_gen_keys(device, n, index, fcw.ctypes.data_as(ctypes.c_void_p), p, nq,
                                   seeds.ctypes.data_as(ctypes.c_void_p),
                                   out.ctypes.data_as(ctypes.c_void_p)), "pir_gen_keys")
    return [out[j * kl:(j + 1) * kl].tobytes() for j in range(p)]
