"""ctypes binding of the C ABI declared in include/smallz4_amd.h.

The product path is the in-tree HIP library ``smallz4_amd/lib/libsmallz4_amd.so``
(built by ``__graft_entry__.build()``).  There is no fallback: if the library is
missing or no GPU is visible, every compression call raises.
"""
from __future__ import annotations

import ctypes
import os

LIB_PATH = os.environ.get("SMALLZ4_AMD_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib",
                                                               "libsmallz4_amd.so")

SZ4_OK = 0
SZ4_E_CAPACITY = -3
SZ4_E_CORRUPT = -6
SZ4_HEADER_SMALLZ4 = 0
SZ4_HEADER_INDEPENDENT = 1
SZ4_HEADER_NONE = 2

# every symbol include/smallz4_amd.h declares, with its ctypes signature
_u64, _u32, _i32, _vp = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p
# the reference's callback types (smallz4.h:41-44, smallz4cat.c:62-65)
GET_BYTES = ctypes.CFUNCTYPE(ctypes.c_size_t, _vp, ctypes.c_size_t, _vp)
SEND_BYTES = ctypes.CFUNCTYPE(None, _vp, ctypes.c_size_t, _vp)
GET_BYTE = ctypes.CFUNCTYPE(ctypes.c_ubyte, _vp)
SEND_OUT = ctypes.CFUNCTYPE(None, ctypes.POINTER(ctypes.c_ubyte), ctypes.c_uint, _vp)
SIGNATURES = {
    "sz4_version": (ctypes.c_char_p, []),
    "sz4_create": (_i32, [ctypes.POINTER(_vp), _i32, _u64]),
    "sz4_destroy": (None, [_vp]),
    "sz4_acquire": (_i32, [ctypes.POINTER(_vp), _i32]),
    "sz4_release": (None, [_vp]),
    "sz4_bound": (_u64, [_u64, _u32]),
    "sz4_compress_blocks_device": (_i32, [_vp, _vp, _u64, _u32, _u32, _i32, _vp, _u64, ctypes.POINTER(_u64), _vp]),
    "sz4_last_block_sizes": (ctypes.c_int64, [_vp, ctypes.POINTER(_u32), _u64]),
    "sz4_lz4": (_i32, [_vp, _vp, _u64, _u32, _vp, _u64, _i32, _vp, _u64, ctypes.POINTER(_u64)]),
    "sz4_lz4_bound": (_u64, [_u64, _i32]),
    "sz4_lz4_stream": (_i32, [_vp, GET_BYTES, SEND_BYTES, _u32, _vp, _u64, _i32, _vp]),
    "sz4_set_stream_chunk": (None, [_vp, _u64]),
    "sz4_set_batch_chunk": (None, [_vp, _u64]),
    "sz4_unlz4_stream": (_i32, [_vp, GET_BYTE, SEND_OUT, _vp, _u64, _vp]),
    "sz4_last_stage_ms": (_i32, [_vp, ctypes.POINTER(ctypes.c_float), _i32]),
    "sz4_set_timing": (None, [_vp, _i32]),
    "sz4_debug_stop_after": (None, [_vp, _i32]),
    "sz4_debug_matches": (_i32, [_vp, _vp, _vp, _u64]),
    "sz4_unlz4": (_i32, [_vp, _vp, _u64, _vp, _u64, _vp, _u64, ctypes.POINTER(_u64)]),
    "sz4_unlz4_device": (_i32, [_vp, _vp, _u64, _vp, _u64, _vp, _u64, ctypes.POINTER(_u64), _vp]),
    "sz4_device_bytes": (_u64, [_vp]),
    "sz4_trim": (None, [_vp]),
    "sz4_set_device_limit": (None, [_vp, _u64]),
    "sz4_released_buffers": (_u64, [_vp]),
    "sz4_set_pool_cap": (None, [_u64]),
    "sz4_dict_rounds": (_u32, [_vp]),
    "sz4_unlz4_resolve_passes": (_u32, [_vp]),
    "sz4_unlz4_index_parallel": (_i32, [_vp]),
    "sz4_last_error": (ctypes.c_char_p, [_vp]),
}

_lib = None


class NativeError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    """Load the HIP library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        # torch (device memory, streams) bundles its own libamdhip64.so.7; load it first so the
        # library binds to the same HIP runtime instead of a second copy from /opt/rocm
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise NativeError(f"{LIB_PATH} is missing: run __graft_entry__.build() (hipcc, gfx950)")
        l = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        _lib = l
    return _lib
