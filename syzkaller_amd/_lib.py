"""ctypes binding of libsyzsig.so (the C ABI declared in include/syzsig.h).

The library is built in-tree (``make`` -> ``syzkaller_amd/libsyzsig.so``).
There is no fallback: if it is missing, importing the GPU API raises.
"""
import ctypes
import os
from ctypes import POINTER, c_char_p, c_int, c_int8, c_uint8, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SYZSIG_LIB") or os.path.join(_HERE, "libsyzsig.so")  # SYZSIG_LIB: an experiment build

SYZSIG_OK = 0
SYZSIG_EIO = -5
SYZSIG_ENOMEM = -12
SYZSIG_EINVAL = -22
SYZSIG_ERANGE = -34
SYZSIG_ECORRUPT = -74
SYZSIG_DEBUG_FIN_DEFER = 32
SYZSIG_DEBUG_MIN_ATOMIC = 64
SYZSIG_DEBUG_EXACT_CELLS = 128
SYZSIG_DEBUG_CAP_SPILL = 256
SYZSIG_DEBUG_RECS_GATE = 512
SYZSIG_DEBUG_EDGE_MARKALL = 1024
SYZSIG_DEBUG_EDGE_PASSES = 2048
SYZSIG_DEBUG_POLL_FAIL = 4096
SYZSIG_DEBUG_AGG_IDX64 = 8192


class SyzsigError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"syzsig error {code}: {msg}")
        self.code = code


class CorruptedSerial(SyzsigError):
    """panic("corrupted Serial") of pkg/signal/signal.go:60-62."""


class SynthCfg(ctypes.Structure):
    _fields_ = [("seed", c_uint64), ("nblocks_log2", c_uint32), ("region_log2", c_uint32),
                ("nsys", c_uint32), ("skew", c_uint32), ("restart_log2", c_uint32),
                ("errno_permille", c_uint32), ("any_permille", c_uint32), ("bad_pc_ppm", c_uint32),
                ("global_walk", c_uint32)]


class Batch(ctypes.Structure):
    _fields_ = [("sigs", c_void_p), ("call_start", c_void_p), ("call_len", c_void_p),
                ("call_prio", c_void_p), ("ncalls", c_uint64), ("nrec", c_uint64),
                ("new_bits", c_void_p), ("call_new", c_void_p), ("new_pairs", c_void_p),
                ("new_pairs_cap", c_uint64)]


class BatchStats(ctypes.Structure):
    _fields_ = [("records", c_uint64), ("survivors", c_uint64), ("candidates", c_uint64), ("changed", c_uint64),
                ("inserted", c_uint64), ("new_signal_len", c_uint64), ("retries", c_uint64),
                ("runs", c_uint64), ("parts", c_uint64), ("distinct", c_uint64), ("overflow_parts", c_uint64),
                ("new_pairs", c_uint64), ("part_ms", ctypes.c_double), ("probe_ms", ctypes.c_double), ("decide_ms", ctypes.c_double)]

    def as_dict(self):
        return {f[0]: (float if f[1] is ctypes.c_double else int)(getattr(self, f[0])) for f in self._fields_}


class StepStatus(ctypes.Structure):
    """syzsig_step_status: what syzsig_step_finish reports for one sharded step."""
    _fields_ = [("src_void", c_uint64), ("global_void", c_uint64), ("owners_void", c_uint64), ("records", c_uint64),
                ("distinct", c_uint64), ("sent", c_uint64), ("max_out", c_uint64), ("received", c_uint64),
                ("max_in", c_uint64), ("own_distinct", c_uint64), ("inserted", c_uint64), ("changed", c_uint64),
                ("new_pairs", c_uint64), ("own_parts", c_uint64), ("src_ms", ctypes.c_double),
                ("own_ms", ctypes.c_double), ("back_ms", ctypes.c_double)]

    def as_dict(self):
        return {f[0]: (float if f[1] is ctypes.c_double else int)(getattr(self, f[0])) for f in self._fields_}


STEP_HDR_VOID = 1 << 63
STEP_HDR_OVF = 1 << 62
STEP_HDR_COUNT = (1 << 40) - 1

_P = c_void_p
_PP = POINTER(c_void_p)

# name -> (restype, argtypes); must cover every function of include/syzsig.h
SIGNATURES = {
    "syzsig_abi_version": (c_int, []),
    "syzsig_last_error": (c_char_p, []),
    "syzsig_ctx_create": (c_int, [c_int, _PP]),
    "syzsig_ctx_destroy": (None, [_P]),
    "syzsig_ctx_set_stream": (c_int, [_P, _P]),
    "syzsig_ctx_stream": (_P, [_P]),
    "syzsig_ctx_set_timing": (c_int, [_P, c_int]),
    "syzsig_ctx_set_agg": (c_int, [_P, c_int, ctypes.c_uint32]),
    "syzsig_ctx_set_debug": (c_int, [_P, ctypes.c_uint32]),
    "syzsig_ctx_last_ms": (ctypes.c_double, [_P]),
    "syzsig_copy_bw_dev": (c_int, [_P, _P, _P, c_uint64, POINTER(ctypes.c_double)]),
    "syzsig_host_alloc": (c_int, [_P, c_uint64, POINTER(_P)]),
    "syzsig_host_free": (c_int, [_P, _P]),
    "syzsig_set_make": (c_int, [_P, c_uint64, _PP]),
    "syzsig_set_free": (None, [_P]),
    "syzsig_set_clone": (c_int, [_P, _P, _PP]),
    "syzsig_set_clear": (c_int, [_P, _P]),
    "syzsig_set_copy_from": (c_int, [_P, _P, _P]),
    "syzsig_set_restore_keys": (c_int, [_P, _P, _P, _P]),
    "syzsig_set_equal": (c_int, [_P, _P, _P, ctypes.POINTER(c_int)]),
    "syzsig_set_reserve": (c_int, [_P, _P, c_uint64]),
    "syzsig_len": (c_uint64, [_P]),
    "syzsig_empty": (c_int, [_P]),
    "syzsig_capacity": (c_uint64, [_P]),
    "syzsig_from_raw": (c_int, [_P, _P, c_uint64, c_uint8, _PP]),
    "syzsig_serialize": (c_int, [_P, _P, _P, _P, c_uint64, POINTER(c_uint64)]),
    "syzsig_serialize_batch": (c_int, [_P, _P, c_uint64, _P, _P, c_uint64, _P]),
    "syzsig_deserialize": (c_int, [_P, _P, c_uint64, _P, c_uint64, _PP]),
    "syzsig_deserialize_dev": (c_int, [_P, _P, _P, c_uint64, _PP]),
    "syzsig_diff": (c_int, [_P, _P, _P, _PP]),
    "syzsig_diff_raw": (c_int, [_P, _P, _P, c_uint64, c_uint8, _PP]),
    "syzsig_intersection": (c_int, [_P, _P, _P, _PP]),
    "syzsig_merge": (c_int, [_P, _PP, _P]),
    "syzsig_manager_poll_batch": (c_int, [_P, _PP, _P, c_uint32, _P, _P, _P, _P, c_uint32, _P]),
    "syzsig_cover_merge": (c_int, [_P, _PP, _P, c_uint64]),
    "syzsig_cover_merge_dev": (c_int, [_P, _PP, _P, c_uint64]),
    "syzsig_triage_runs_dev": (c_int, [_P, _P, c_uint64, _P, _P, _P, ctypes.c_uint32, _P, _P, _P, _P, _P, _P, _P]),
    "syzsig_minimize_pred_dev": (c_int, [_P, _P, c_uint64, _P, _P, _P, ctypes.c_uint32, _P, _P, _P, _P, _P, _P]),
    "syzsig_minimize": (c_int, [_P, _P, _P, _P, c_uint64, c_uint64, _P, POINTER(c_uint64)]),
    "syzsig_minimize_dev": (c_int, [_P, _P, _P, _P, c_uint64, c_uint64, _P, POINTER(c_uint64)]),
    "syzsig_minimize_shard_dev": (c_int, [_P, _P, _P, _P, c_uint64, c_uint32, c_uint32, c_uint64, _P, POINTER(c_uint64)]),
    "syzsig_minimize_split_dev": (c_int, [_P, _P, _P, _P, c_uint64, c_uint32, c_uint32, c_uint32, c_uint64, _P,
                                          c_uint64, _P]),
    "syzsig_minimize_resolve_dev": (c_int, [_P, _P, c_uint64, _P, c_uint64, _P, POINTER(c_uint64)]),
    "syzsig_check_new_signal": (c_int, [_P, _PP, _PP, _P, c_uint64, _P, _P, _P, c_uint32, _P,
                                        POINTER(c_uint32), _P]),
    "syzsig_triage_batch": (c_int, [_P, _P, _PP, POINTER(Batch), POINTER(BatchStats)]),
    "syzsig_edge_derive_dev": (c_int, [_P, _P, c_uint64, _P, _P, c_uint64, _P, c_uint64, _P, _P, _P]),
    "syzsig_ingest_exec_output_dev": (c_int, [_P, _P, c_uint64, _P, c_uint64, _P, c_uint64, _P, _P, _P, _P, _P, _P,
                                              _P, _P, _P, POINTER(c_uint64)]),
    "syzsig_triage_records_dev": (c_int, [_P, _P, _PP, _P, c_uint64, _P, c_uint32, _P,
                                          POINTER(BatchStats)]),
    "syzsig_step_send_dev": (c_int, [_P, POINTER(Batch), c_uint64, _P, c_uint32, c_uint32, c_uint64, _P, c_int]),
    "syzsig_step_own_dev": (c_int, [_P, _P, _P, _P, c_uint32, c_uint64, _P, c_uint32, _P, c_int]),
    "syzsig_step_back_dev": (c_int, [_P, POINTER(Batch), c_uint64, _P, c_uint32, c_uint64, _P]),
    "syzsig_step_finish": (c_int, [_P, POINTER(StepStatus)]),
    "syzsig_synth_default": (None, [POINTER(SynthCfg)]),
    "syzsig_synth_traces_host": (c_int, [POINTER(SynthCfg), c_uint64, c_uint64, c_uint32, _P, _P, _P, _P]),
    "syzsig_synth_traces_dev": (c_int, [_P, POINTER(SynthCfg), c_uint64, c_uint64, c_uint32, _P, _P, _P, _P]),
    "syzsig_synth_m0_host": (c_int, [POINTER(SynthCfg), c_uint64, c_uint64, _P, _P]),
    "syzsig_synth_m0_dev": (c_int, [_P, POINTER(SynthCfg), c_uint64, c_uint64, _P, _P]),
    "syzsig_synth_m0_shard_dev": (c_int, [_P, POINTER(SynthCfg), c_uint64, c_uint64, c_uint32, c_uint32, _P, _P,
                                          c_uint64, POINTER(c_uint64)]),
}

_lib = None


def lib():
    """Load libsyzsig.so (raises if it was not built: there is no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `make` (or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc):
    if rc != SYZSIG_OK:
        msg = lib().syzsig_last_error().decode(errors="replace")
        if rc == SYZSIG_ECORRUPT:
            raise CorruptedSerial(rc, msg)
        raise SyzsigError(rc, msg)
    return rc


def synth_default(**over):
    c = SynthCfg()
    lib().syzsig_synth_default(ctypes.byref(c))
    for k, v in over.items():
        setattr(c, k, v)
    return c
