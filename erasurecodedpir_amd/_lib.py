"""ctypes binding of libpir_engine.so (the C ABI declared in include/pir_engine.h,
include/pir_server.h and include/pir_client.h).

The library is built in-tree (erasurecodedpir_amd/libpir_engine.so, see csrc/Makefile and
__graft_entry__.build()).  There is no fallback: if the library is missing or a GPU call
fails, the error propagates.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# $PIR_ENGINE_LIB: another build of the same library (A/B diagnostics only)
LIB_PATH = os.environ.get("PIR_ENGINE_LIB") or os.path.join(_HERE, "libpir_engine.so")

c_u8_p = ctypes.POINTER(ctypes.c_uint8)


class PirConfig(ctypes.Structure):
    _fields_ = [
        ("device", ctypes.c_int),
        ("num_parties", ctypes.c_int),
        ("party_index", ctypes.c_int),
        ("log_num_records", ctypes.c_int),
        ("record_bytes", ctypes.c_uint32),
        ("num_rounds", ctypes.c_int),
        ("log_num_partitions", ctypes.c_int),
        ("partition_index", ctypes.c_int),
        ("is_byzantine", ctypes.c_int),
    ]


class PirCommInfo(ctypes.Structure):  # pir_comm_info_t (include/pir_engine.h)
    _fields_ = [
        ("attached", ctypes.c_int),
        ("count", ctypes.c_int),
        ("user_rank", ctypes.c_int),
        ("device", ctypes.c_int),
        ("engine_device", ctypes.c_int),
        ("pci_bus_id", ctypes.c_char * 64),
    ]


class PirKernelTime(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 32), ("ms", ctypes.c_float)]


class CServer(ctypes.Structure):  # include/pir_server.h `server` (src/c/server.h:13-25)
    _fields_ = [
        ("ctx", ctypes.c_void_p),
        ("ctxThreads", ctypes.c_void_p),
        ("partyIndex", ctypes.c_int),
        ("indexList", ctypes.POINTER(c_u8_p)),
        ("isByzantine", ctypes.c_int),
        ("numThreads", ctypes.c_int),
    ]


class CClient(ctypes.Structure):  # include/pir_server.h `client` (src/c/client.h:15-20)
    _fields_ = [
        ("ctx", ctypes.c_void_p),
        ("macCtx", ctypes.c_void_p),
        ("unencoded_files", ctypes.POINTER(c_u8_p)),
        ("macKey", c_u8_p),
    ]


# name -> (restype, argtypes)
class U128(ctypes.Structure):  # uint128_t (utils.h:13-15) by value: two INTEGER eightbytes
    _fields_ = [("lo", ctypes.c_uint64), ("hi", ctypes.c_uint64)]


_P = ctypes.c_void_p
_I = ctypes.c_int
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
_SZ = ctypes.c_size_t
PROTOTYPES = {
    # pir_engine.h
    "pir_engine_last_error": (ctypes.c_char_p, []),
    "pir_engine_create": (_I, [ctypes.POINTER(PirConfig), ctypes.POINTER(_P)]),
    "pir_engine_destroy": (None, [_P]),
    "pir_engine_key_len": (_I, [_I, _I, _I]),
    "pir_engine_num_rows": (_U64, [_P]),
    "pir_engine_set_shard": (_I, [_P, _P, _U64, _U64, _U64]),
    "pir_engine_set_shard_rows": (_I, [_P, _P, _U64, _U64]),
    "pir_engine_get_shard_rows": (_I, [_P, _P, _U64, _U64]),
    "pir_engine_encode_across_rows": (_I, [_P, _P, _U64, _I]),
    "pir_engine_encode_within_rows": (_I, [_P, _P, _U64, ctypes.c_uint32, _I, _I]),
    "pir_engine_fill_shard_random": (_I, [_P, _U64]),
    "pir_engine_encode_across_dev": (_I, [_P, _P, _U64, _U64, _I]),
    "pir_engine_encode_within_dev": (_I, [_P, _P, _U64, _U64, ctypes.c_uint32, _I, _I]),
    "pir_engine_get_shard_row": (_I, [_P, _U64, _P]),
    "pir_engine_get_shard": (_I, [_P, _U64, _U64, _P]),
    "pir_engine_answer": (_I, [_P, _P, _P]),
    "pir_engine_answer_slice": (_I, [_P, _P, _I, _I, _P]),
    "pir_engine_answer_slices": (_I, [_P, _P, _I, _P]),
    "pir_engine_answer_slices_dev": (_I, [_P, _P, _I, _P, _P]),
    "pir_engine_fold_gathered_dev": (_I, [_P, _P, _I, ctypes.c_uint64, _P, _P]),
    "pir_engine_eval_all": (_I, [_P, _P, _P]),
    "pir_engine_answer_coefs": (_I, [_P, ctypes.POINTER(_P), _U64, _U64, _P]),
    "pir_engine_answer_coefs_dev": (_I, [_P, _P, _U64, _U64, _U64, _P, _P]),
    "pir_engine_answer_mp": (_I, [_P, _P, _U64, _I, _I, _I, _I, _P]),
    "pir_engine_answer_mp_dev": (_I, [_P, _P, _I, _I, _I, _I, _P, _P]),
    "pir_engine_mp_num_keys": (_I, [_I, _I]),
    "pir_engine_mp_key_len": (_I, [_I, _I, _I]),
    "pir_engine_answer_cd": (_I, [_P, _P, _U64, _I, _I, _I, _I, _P]),
    "pir_engine_answer_cd_dev": (_I, [_P, _P, _I, _I, _I, _I, _P, _P]),
    "pir_engine_cd_key_len": (_I, [_I, _I, _I, _I, _I]),
    "pir_engine_mp_eval_bytes": (ctypes.c_longlong, [_I, _I, _I]),
    "pir_engine_answer_dev": (_I, [_P, _P, _P, _P]),
    "pir_engine_answer_batch_dev": (_I, [_P, _P, _I, _P, _P]),
    "pir_engine_answer_batch": (_I, [_P, _P, _I, _P]),
    "pir_engine_answer_stream_dev": (_I, [_P, _P, _I, _P, _P]),
    "pir_engine_reserve_queue": (_I, [_P, _I]),
    "pir_engine_set_batch_group": (_I, [_P, _I]),
    "pir_engine_batch_group": (_I, [_P]),
    "pir_engine_stream": (_P, [_P]),
    "pir_engine_sync": (_I, [_P]),
    "pir_engine_alloc_dev": (_I, [_P, _SZ, ctypes.POINTER(_P)]),
    "pir_engine_free_dev": (_I, [_P, _P]),
    "pir_engine_set_party_index": (_I, [_P, _I]),
    "pir_engine_memcpy_h2d": (_I, [_P, _P, _P, _SZ]),
    "pir_engine_memcpy_d2h": (_I, [_P, _P, _P, _SZ]),
    "pir_engine_set_profiling": (_I, [_P, _I]),
    "pir_engine_last_timings": (_I, [_P, ctypes.POINTER(PirKernelTime), _I]),
    "pir_engine_profile_phases": (_I, [_P, _P, _I, ctypes.POINTER(ctypes.c_float)]),
    "pir_engine_trace_query": (_I, [_P, _P, _I, _P, _I]),
    "pir_comm_unique_id": (_I, [_P]),
    "pir_comm_attach": (_I, [_P, _P, _I, _I]),
    "pir_comm_detach": (_I, [_P]),
    "pir_comm_info": (_I, [_P, ctypes.POINTER(PirCommInfo)]),
    # pir_client.h
    "pir_gen_keys": (_I, [_I, _I, _U64, _P, _I, _I, _P, _P]),
    "pir_final_cw": (None, [_I, _I, _I, _P]),
    # pir_server.h (reference names)
    "setSystemParams": (None, [_I, _I, _I, _I, _I, _I, _I, _I, _I]),
    "freeParams": (None, []),
    "calcOptimizedDPFTreeKeyLength": (_I, [_I, _I, _I]),
    "initializeServer": (None, [ctypes.POINTER(CServer), _I, _U32, _U32, _I, _I]),
    "freeServer": (None, [ctypes.POINTER(CServer)]),
    "runOptimizedDPFTreeQuery": (None, [ctypes.POINTER(CServer), _P, _I, ctypes.POINTER(c_u8_p)]),
    "runOptimizedDPFTreeQueryThread": (None, [ctypes.POINTER(CServer), _P, _I, _I,
                                              ctypes.POINTER(c_u8_p)]),
    "assemblDPFTreeQueryThreadResults": (None, [ctypes.POINTER(CServer),
                                                ctypes.POINTER(ctypes.POINTER(c_u8_p)), _I,
                                                ctypes.POINTER(c_u8_p)]),
    "initialize_client": (None, [ctypes.POINTER(CClient), ctypes.c_uint8, _U32]),
    "free_client": (None, [ctypes.POINTER(CClient)]),
    "encode_across_files_server": (None, [ctypes.POINTER(CClient), ctypes.POINTER(CServer)]),
    "assembleDPFTreeQueryResponses": (None, [ctypes.POINTER(CClient), _P,
                                             ctypes.POINTER(ctypes.POINTER(c_u8_p)), _P]),
    "assembleHollantiResponses": (None, [ctypes.POINTER(CClient), _P,
                                         ctypes.POINTER(ctypes.POINTER(c_u8_p)), _P]),
    "lagrangeInterpolationSemihonest": (None, [_P, ctypes.c_uint8, _P, ctypes.c_uint8, _P]),
    "runHollantiQuery": (None, [ctypes.POINTER(CServer), ctypes.POINTER(c_u8_p),
                                ctypes.POINTER(c_u8_p)]),
    "runHollantiQueryThread": (None, [ctypes.POINTER(CServer), ctypes.POINTER(c_u8_p), _I, _I, _I,
                                      ctypes.POINTER(c_u8_p)]),
    "assembleHollantiQueryThreadResults": (None, [ctypes.POINTER(CServer),
                                                  ctypes.POINTER(ctypes.POINTER(c_u8_p)), _I,
                                                  ctypes.POINTER(c_u8_p)]),
    "encode_within_files_server": (None, [ctypes.POINTER(CClient), ctypes.POINTER(CServer)]),
    "runOptShamirDPFQueryThread": (None, [ctypes.POINTER(CServer), ctypes.POINTER(c_u8_p), _I, _I,
                                          _I, ctypes.POINTER(c_u8_p)]),
    "calcMultiPartyOptDPFKeyLength": (_I, [_I, _I, _I]),
    "runOptimizedMultiPartyDPFQuery": (None, [ctypes.POINTER(CServer), _P, ctypes.POINTER(c_u8_p)]),
    "runOptimizedMultiPartyDPFQueryThread": (None, [ctypes.POINTER(CServer), _P, _I, _I,
                                                    ctypes.POINTER(c_u8_p)]),
    "runCDQueryThread": (None, [ctypes.POINTER(CServer), _P, _I, _I, ctypes.POINTER(c_u8_p)]),
    "runWoodruffQueryThread": (None, [ctypes.POINTER(CServer), _P, _I, _I, _I,
                                      ctypes.POINTER(c_u8_p)]),
    "assembleShamirQueryThreadResults": (None, [ctypes.POINTER(CServer),
                                                ctypes.POINTER(ctypes.POINTER(c_u8_p)), _I,
                                                ctypes.POINTER(c_u8_p)]),
    "assembleMultipartyDPFQueryThreadResults": (None, [ctypes.POINTER(CServer),
                                                       ctypes.POINTER(ctypes.POINTER(c_u8_p)), _I,
                                                       ctypes.POINTER(c_u8_p)]),
    "assembleCDQueryThreadResults": (None, [ctypes.POINTER(CServer),
                                            ctypes.POINTER(ctypes.POINTER(c_u8_p)), _I,
                                            ctypes.POINTER(c_u8_p)]),
    "assembleWoodruffQueryThreadResults": (None, [ctypes.POINTER(CServer),
                                                  ctypes.POINTER(ctypes.POINTER(c_u8_p)), _I,
                                                  ctypes.POINTER(c_u8_p)]),
    "calcShamirDPFKeyLength": (_I, [_I]),
    "calcShamirResponseLength": (_I, [_I, _I]),
    # client-side names of package c (src/client, src/benchmark)
    "generate_opt_DPF_tree_query": (None, [ctypes.POINTER(CClient), _I,
                                           ctypes.POINTER(ctypes.POINTER(c_u8_p))]),
    "generateHollantiQuery": (None, [ctypes.POINTER(CClient), _I,
                                     ctypes.POINTER(ctypes.POINTER(c_u8_p))]),
    "mac": (None, [_P, _P, _I, _P, _I]),
    "choose": (_I, [_I, _I]),
    "convertInt": (U128, [_I]),
    "calcCDDPFKeyLength": (_I, [_I, _I, _I, _I, _I]),
    "calcWoodruffKeyLength": (_I, [_I, _I, _I, _I, _I]),
    "generateMultiPartyDPFQuery": (None, [ctypes.POINTER(CClient), _I,
                                          ctypes.POINTER(ctypes.POINTER(c_u8_p))]),
    "assembleMultiPartyResponses": (None, [ctypes.POINTER(CClient), _P,
                                           ctypes.POINTER(ctypes.POINTER(c_u8_p)), _P]),
    "generateCDQuery": (None, [ctypes.POINTER(CClient), _I,
                               ctypes.POINTER(ctypes.POINTER(c_u8_p))]),
    "assembleCDResponses": (None, [ctypes.POINTER(CClient), _P,
                                   ctypes.POINTER(ctypes.POINTER(c_u8_p)), _P]),
    "genShamirCoeffs": (None, [_I, _I, _I, U128, _P, _P]),
    "genOptShamirDPF": (None, [_I, U128, _I, _I, _I, _P, _P, _P]),
    "assembleShamirResponses": (None, [ctypes.POINTER(CClient), _P, _P, _P, _P, _P]),
    "genWoodruffVs": (None, [_I, _I, _P]),
    "genWoodruffQuery": (None, [U128, _I, _I, _I, _P, _P]),
    "assembleWoodruffResponses": (None, [ctypes.POINTER(CClient), _P, _P, _P, _P]),
    "pirSetDevice": (None, [_I]),
    "pirServerShardChanged": (None, [ctypes.POINTER(CServer)]),
    "pirServerSyncRows": (None, [ctypes.POINTER(CServer)]),
    "pirRunTreeQueryThreads": (None, [ctypes.POINTER(CServer), ctypes.c_void_p, ctypes.c_int,
                                      ctypes.c_void_p]),
    "pirServerSetRows": (None, [ctypes.POINTER(CServer), ctypes.c_void_p, ctypes.c_uint64,
                                ctypes.c_uint64, ctypes.c_uint32]),
    "pirServerWaitFreed": (None, []),
}

GLOBALS_INT = ["NUM_PARTIES", "NUM_FILES", "NUM_ENCODED_FILES", "LOG_NUM_ENCODED_FILES",
               "ENCODED_PAYLOAD_SIZE_BYTES", "ENCODED_FILE_SIZE_BYTES", "ENCODE_ACROSS",
               "NUM_ROUNDS", "RHO", "K", "T", "R", "B", "NUM_RESPONSES", "MODE", "IS_HERMITE",
               "D", "MAC_SIZE_BYTES", "CHECK_MAC", "NUM_RSS_KEYS", "NUM_CD_KEYS",
               "NUM_CD_KEYS_NEEDED", "WOODRUFF_M",
               "WOODRUFF_D", "WOODRUFF_DERIVATIVE"]
GLOBALS_U32 = ["LOG_NUM_FILES", "FILE_SIZE_BYTES", "PAYLOAD_SIZE_BYTES"]

_lib = None


def load():
    """Load libpir_engine.so; raises OSError when it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OSError(f"{LIB_PATH} not built: run `make -C erasurecodedpir_amd/csrc` or "
                      "__graft_entry__.build()")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in PROTOTYPES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def global_int(name):
    lib = load()
    t = ctypes.c_uint32 if name in GLOBALS_U32 else ctypes.c_int
    return t.in_dll(lib, name).value


class PirError(RuntimeError):
    pass


def check(rc, what):
    if rc != 0:
        msg = load().pir_engine_last_error()
        raise PirError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
