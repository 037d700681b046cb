"""MI355X-native tree-DPF PIR server-answer engine.

The hot path -- full-domain DPF evaluation (AES-128 PRG tree) followed by the GF(2^8)
inner product against the device-resident shard -- runs as hand-written HIP kernels for
gfx950 in libpir_engine.so, behind a C ABI (include/pir_engine.h) and a drop-in for the
reference's server.h entry points (include/pir_server.h).
"""
from ._lib import LIB_PATH, PirError, load  # noqa: F401
from .client import final_cw, gen_keys  # noqa: F401
from .engine import Engine, cd_key_len, comm_unique_id, key_len, mp_eval_bytes, mp_key_len, mp_num_keys  # noqa: F401

__all__ = ["Engine", "gen_keys", "final_cw", "key_len", "mp_num_keys", "mp_key_len", "mp_eval_bytes", "cd_key_len", "comm_unique_id", "load", "LIB_PATH",
           "PirError"]
