"""ctypes binding of the C-ABI in include/lora_mi355x.h (liblora_mi355x.so).

The shared library is built in-tree (``make -C lora-sdr-lightweight-standalone-library-_amd``
or ``__graft_entry__.build()``) into ``lora_phy_amd/lib/``.  There is no CPU fallback:
if the library or a GPU is missing, the product API raises.
"""
from __future__ import annotations

import ctypes as C
import os

# LORA_MI355X_LIB: development A/B of an alternative in-tree build of the same library.
LIB_PATH = os.environ.get("LORA_MI355X_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib",
                                                             "liblora_mi355x.so")

LORA_OK = 0
LORA_EIO = -5
LORA_ENOMEM = -12
LORA_EINVAL = -22
LORA_ERANGE = -34

LORA_WINDOW_NONE = 0
LORA_WINDOW_HANN = 1
LORA_MODE_LEGACY = 0
LORA_MODE_API = 1
LORA_MODE_RAW = 2

# lora_demod_last_kernels bits
KERNEL_BITS = {"frame_max": 1, "estimate": 2, "demod": 4, "generic": 16, "frame_max_wave": 32, "spec": 64}

# Every symbol include/lora_mi355x.h declares (checked by tests/test_capi_symbols.py).
EXPORTED_SYMBOLS = (
    "lora_demod_plan_create",
    "lora_demod_plan_destroy",
    "lora_demod_symbols_per_frame",
    "lora_demod_workspace_bytes",
    "lora_demod_batch",
    "lora_mod_batch",
    "lora_estimate_offsets_batch",
    "lora_compensate_offsets_batch",
    "lora_demod_profile_enable",
    "lora_demod_profile_read",
    "lora_demod_last_kernels",
    "lora_demod_spec_recomputed",
    "lora_demod_plan_set_pipeline",
    "lora_aql_last_profile",
    "lora_last_error",
    "lora_version",
)


class DemodParams(C.Structure):
    _fields_ = [
        ("sf", C.c_uint),
        ("osr", C.c_uint),
        ("bw_hz", C.c_uint),
        ("window", C.c_int),
        ("dechirp", C.c_int),
        ("mode", C.c_int),
        ("device", C.c_int),
        ("precision", C.c_int),
    ]


class DemodOutputs(C.Structure):
    _fields_ = [
        ("symbols", C.c_void_p),
        ("sym_stride", C.c_int64),
        ("sync", C.c_void_p),
        ("cfo", C.c_void_p),
        ("time_offset", C.c_void_p),
        ("max_amp", C.c_void_p),
    ]


class LoraError(RuntimeError):
    """Raised for negative return codes of the C-ABI (reference: -1 / 0 returns)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"{msg} (code {code})")
        self.code = code


_lib = None


def lib() -> C.CDLL:
    """Load liblora_mi355x.so once; raise loudly if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build the HIP extension first "
            "(python -c 'import __graft_entry__ as g; g.build()')")
    L = C.CDLL(LIB_PATH)
    L.lora_demod_plan_create.restype = C.c_int
    L.lora_demod_plan_create.argtypes = [C.POINTER(DemodParams), C.POINTER(C.c_void_p)]
    L.lora_demod_plan_destroy.restype = C.c_int
    L.lora_demod_plan_destroy.argtypes = [C.c_void_p]
    L.lora_demod_symbols_per_frame.restype = C.c_int64
    L.lora_demod_symbols_per_frame.argtypes = [C.c_void_p, C.c_int64]
    L.lora_demod_workspace_bytes.restype = C.c_size_t
    L.lora_demod_workspace_bytes.argtypes = [C.c_void_p, C.c_int64, C.c_int64]
    L.lora_demod_batch.restype = C.c_int64
    L.lora_demod_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_int64,
                                   C.POINTER(DemodOutputs), C.c_void_p, C.c_size_t, C.c_void_p]
    L.lora_mod_batch.restype = C.c_int64
    L.lora_mod_batch.argtypes = [C.c_uint, C.c_uint, C.c_uint, C.c_float, C.c_uint8, C.c_void_p,
                                 C.c_int64, C.c_int64, C.c_void_p, C.c_int, C.c_void_p]
    L.lora_estimate_offsets_batch.restype = C.c_int64
    L.lora_estimate_offsets_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64,
                                              C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]
    L.lora_compensate_offsets_batch.restype = C.c_int64
    L.lora_compensate_offsets_batch.argtypes = [C.c_uint, C.c_uint, C.c_void_p, C.c_int64,
                                                C.c_int64, C.c_int64, C.c_void_p, C.c_void_p,
                                                C.c_int, C.c_void_p, C.c_void_p]
    L.lora_demod_profile_enable.restype = C.c_int
    L.lora_demod_profile_enable.argtypes = [C.c_void_p, C.c_int]
    L.lora_demod_profile_read.restype = C.c_int
    L.lora_demod_profile_read.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_int)]
    L.lora_demod_last_kernels.restype = C.c_int
    L.lora_demod_last_kernels.argtypes = [C.c_void_p]
    L.lora_demod_spec_recomputed.restype = C.c_int64
    L.lora_demod_spec_recomputed.argtypes = [C.c_void_p]
    L.lora_demod_plan_set_pipeline.restype = C.c_int
    L.lora_demod_plan_set_pipeline.argtypes = [C.c_void_p, C.c_int]
    L.lora_aql_last_profile.restype = C.c_int
    L.lora_aql_last_profile.argtypes = [C.POINTER(C.c_double), C.c_int]
    L.lora_last_error.restype = C.c_char_p
    L.lora_version.restype = C.c_char_p
    _lib = L
    return L


def check(rc: int) -> int:
    if rc < 0:
        msg = lib().lora_last_error().decode(errors="replace")
        raise LoraError(int(rc), msg or "lora_mi355x error")
    return int(rc)
