"""ctypes loader for the oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker: the product path never imports it.

  oz_*   : C restatement of the reference (oracle/liboracle.so, always built)
  ref_*  : the reference itself, compiled in place from /root/reference by
           oracle/Makefile (oracle/_ref/libsmallz4_ref.so; absent when the
           reference tree was not available at build time)
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libsmallz4_ref.so")
REF_CAT = os.path.join(HERE, "_ref", "smallz4cat")
REF_CLI = os.path.join(HERE, "_ref", "smallz4")

_C = ctypes
_LZ4_ARGS = [_C.c_char_p, _C.c_uint64, _C.c_uint, _C.c_char_p, _C.c_uint64, _C.c_int, _C.c_char_p, _C.c_uint64]
_o = None
_r = None


def _oracle():
    global _o
    if _o is None:
        if not os.path.exists(ORACLE_SO):
            raise RuntimeError("oracle/liboracle.so missing: run `make -C oracle` (or __graft_entry__.build())")
        l = ctypes.CDLL(ORACLE_SO)
        l.oz_lz4.restype = _C.c_uint64
        l.oz_lz4.argtypes = _LZ4_ARGS
        l.oz_bound.restype = _C.c_uint64
        l.oz_bound.argtypes = [_C.c_uint64, _C.c_int]
        l.oz_block.restype = _C.c_uint64
        l.oz_block.argtypes = [_C.c_char_p, _C.c_uint64, _C.c_uint, _C.c_char_p, _C.c_uint64]
        l.oz_block_matches.restype = None
        l.oz_block_matches.argtypes = [_C.c_char_p, _C.c_uint64, _C.c_uint, _C.c_int, _C.c_void_p, _C.c_void_p]
        l.oz_unlz4.restype = _C.c_uint64
        l.oz_unlz4.argtypes = [_C.c_char_p, _C.c_uint64, _C.c_char_p, _C.c_uint64, _C.c_char_p, _C.c_uint64]
        _o = l
    return _o


def ref_available() -> bool:
    return os.path.exists(REF_SO)


def _ref():
    global _r
    if _r is None:
        l = ctypes.CDLL(REF_SO)
        l.ref_lz4.restype = _C.c_uint64
        l.ref_lz4.argtypes = _LZ4_ARGS
        _r = l
    return _r


def _call(fn, data: bytes, max_chain: int, dictionary: bytes, legacy: bool) -> bytes:
    data = bytes(data)
    cap = _oracle().oz_bound(len(data), int(legacy)) + 4096
    out = ctypes.create_string_buffer(cap)
    dic = bytes(dictionary)
    n = fn(data, len(data), max_chain, dic if dic else None, len(dic), int(legacy), out, cap)
    if n == 0:
        raise RuntimeError("compression failed")
    return out.raw[:n]


def oz_lz4(data: bytes, max_chain: int = 65535, dictionary: bytes = b"", legacy: bool = False) -> bytes:
    """C restatement of smallz4::lz4."""
    return _call(_oracle().oz_lz4, data, max_chain, dictionary, legacy)


def ref_lz4(data: bytes, max_chain: int = 65535, dictionary: bytes = b"", legacy: bool = False) -> bytes:
    """The reference's smallz4::lz4, compiled from /root/reference."""
    return _call(_ref().ref_lz4, data, max_chain, dictionary, legacy)


def oz_block(data: bytes, max_chain: int = 65535) -> bytes:
    """Block word + payload smallz4 emits for `data` compressed on its own."""
    data = bytes(data)
    cap = len(data) + len(data) // 255 + 64
    out = ctypes.create_string_buffer(cap)
    n = _oracle().oz_block(data, len(data), max_chain, out, cap)
    return out.raw[:n]


def oz_unlz4(frame: bytes, dictionary: bytes = b"", cap: int | None = None) -> bytes:
    """Decoder restating smallz4cat (round-trip checks)."""
    frame = bytes(frame)
    if cap is None:
        cap = max(1 << 16, 300 * len(frame))
    out = ctypes.create_string_buffer(cap)
    dic = bytes(dictionary)
    n = _oracle().oz_unlz4(frame, len(frame), dic if dic else None, len(dic), out, cap)
    if n == (1 << 64) - 1:
        raise ValueError("malformed LZ4 frame")
    return out.raw[:n]


def oz_block_matches(data: bytes, max_chain: int, stage: int):
    """(len, dist) numpy arrays of one block at `stage` (see smallz4_oracle.c)."""
    import numpy as np
    data = bytes(data)
    ln = np.zeros(len(data), dtype=np.uint32)
    ds = np.zeros(len(data), dtype=np.uint16)
    _oracle().oz_block_matches(data, len(data), max_chain, stage, ln.ctypes.data, ds.ctypes.data)
    return ln, ds
