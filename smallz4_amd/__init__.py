"""smallz4_amd -- LZ4 optimal-parse compression (smallz4 semantics) on MI355X.

Python mirror of the reference's public interface (reference smallz4.h:38-80):

    smallz4_amd.lz4(data, max_chain_length=65535, dictionary=b"", use_legacy_format=False)
        == bytes the reference's smallz4::lz4(...) emits for `data`
    smallz4_amd.ShortChainsGreedy / ShortChainsLazy / get_version()

plus the data-parallel entry point the GPU is built for:

    Compressor().compress_blocks(data, block_size=65536, max_chain_length=65535)
        -> frame whose every block equals smallz4's output for that block alone

All compression runs in the HIP library smallz4_amd/lib/libsmallz4_amd.so; there
is no CPU fallback.
"""
from __future__ import annotations

import ctypes

from . import _native

ShortChainsGreedy = 3   # smallz4.h:77
ShortChainsLazy = 6     # smallz4.h:79
MaxChainLength = 65535  # smallz4.h:115 ("-9")

# per-stage device timings reported by sz4_last_stage_ms (include/smallz4_amd.h)
STAGES = ("runs", "sort", "find_sorted", "find_long", "parse", "assemble")

HEADERS = {"smallz4": _native.SZ4_HEADER_SMALLZ4, "independent": _native.SZ4_HEADER_INDEPENDENT,
           "none": _native.SZ4_HEADER_NONE}


def get_version() -> str:
    return _native.lib().sz4_version().decode()


def level_to_chain(level: int) -> int:
    """CLI level -0..-9 -> maxChainLength (smallz4.cpp:175, 232-239)."""
    if not 0 <= level <= 9:
        raise ValueError("level must be 0..9")
    return 65535 if level == 9 else level


class Compressor:
    """A device context (HBM scratch stays allocated between calls)."""

    def __init__(self, device: int = 0, reserve_bytes: int = 0):
        self._lib = _native.lib()
        h = ctypes.c_void_p()
        rc = self._lib.sz4_create(ctypes.byref(h), device, reserve_bytes)
        if rc != _native.SZ4_OK:
            raise _native.NativeError(f"sz4_create failed ({rc}): no usable HIP device {device}")
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            self._lib.sz4_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str):
        if rc != _native.SZ4_OK:
            msg = self._lib.sz4_last_error(self._h).decode()
            raise _native.NativeError(f"{what} failed ({rc}): {msg}")

    # -- reference entry point ------------------------------------------------------------------
    def lz4(self, data: bytes, max_chain_length: int = MaxChainLength, dictionary: bytes = b"",
            use_legacy_format: bool = False) -> bytes:
        """Byte-identical to smallz4::lz4 (smallz4.h:47-64) on the same input."""
        data = bytes(data)
        cap = self._lib.sz4_lz4_bound(len(data), int(use_legacy_format))
        out = ctypes.create_string_buffer(cap)
        size = ctypes.c_uint64()
        dic = bytes(dictionary)
        rc = self._lib.sz4_lz4(self._h, data, len(data), int(max_chain_length), dic if dic else None, len(dic),
                               int(use_legacy_format), out, cap, ctypes.byref(size))
        self._check(rc, "sz4_lz4")
        return out.raw[:size.value]

    def lz4_into(self, src, dst, max_chain_length: int = MaxChainLength, dictionary: bytes = b"",
                 use_legacy_format: bool = False) -> int:
        """sz4_lz4 between caller-owned host buffers (numpy uint8 arrays, no Python copies): compresses
        src into dst (at least sz4_lz4_bound(len(src)) bytes) and returns the frame length."""
        import numpy as np
        if isinstance(src, np.ndarray):
            src = np.ascontiguousarray(src, dtype=np.uint8)
        else:  # bytes-like: wrapped without a copy (read-only is fine, the library only reads it)
            src = np.frombuffer(memoryview(src).cast("B"), dtype=np.uint8)
        if not (isinstance(dst, np.ndarray) and dst.dtype == np.uint8 and dst.flags.c_contiguous):
            raise TypeError("dst must be a contiguous numpy uint8 array")
        size = ctypes.c_uint64()
        dic = bytes(dictionary)
        rc = self._lib.sz4_lz4(self._h, ctypes.c_void_p(src.ctypes.data), src.size, int(max_chain_length),
                               dic if dic else None, len(dic), int(use_legacy_format),
                               ctypes.c_void_p(dst.ctypes.data), dst.size, ctypes.byref(size))
        self._check(rc, "sz4_lz4")
        return size.value

    def lz4_stream(self, read, write, max_chain_length: int = MaxChainLength, dictionary: bytes = b"",
                   use_legacy_format: bool = False) -> None:
        """smallz4::lz4 over callbacks (sz4_lz4_stream): read(n) -> bytes (b"" at the end), write(bytes).
        Bounded memory: the input is compressed chunk by chunk (set_stream_chunk)."""
        err = []

        def get(data, n, _user):
            try:
                b = read(n)
            except BaseException as e:  # noqa: BLE001 -- re-raised after the call
                err.append(e)
                return 0
            if b is None:
                return 0
            if len(b) > n:
                # the native buffer holds n bytes: more is a caller error, not a silent overrun
                err.append(ValueError(f"read({n}) returned {len(b)} bytes"))
                return 0
            if b:
                ctypes.memmove(data, b, len(b))
            return len(b)

        def send(data, n, _user):
            try:
                write(ctypes.string_at(data, n) if n else b"")
            except BaseException as e:  # noqa: BLE001
                err.append(e)

        g, s = _native.GET_BYTES(get), _native.SEND_BYTES(send)
        dic = bytes(dictionary)
        rc = self._lib.sz4_lz4_stream(self._h, g, s, int(max_chain_length), dic if dic else None, len(dic),
                                      int(use_legacy_format), None)
        if err:
            raise err[0]
        self._check(rc, "sz4_lz4_stream")

    def set_stream_chunk(self, nbytes: int):
        """Input bytes per chunk of the stream paths (whole blocks; 0 = default 64 MiB)."""
        self._lib.sz4_set_stream_chunk(self._h, int(nbytes))

    def set_batch_chunk(self, nbytes: int):
        """Input bytes per internal piece of compress_blocks(_device) (whole blocks; 0 = default 448 MiB)."""
        self._lib.sz4_set_batch_chunk(self._h, int(nbytes))

    # -- data-parallel entry point --------------------------------------------------------------
    def compress_blocks_device(self, d_in: int, n: int, d_out: int, out_cap: int, block_size: int = 65536,
                               max_chain_length: int = MaxChainLength, header: str = "smallz4",
                               stream: int = 0) -> int:
        """Device pointers in, frame size out (see sz4_compress_blocks_device)."""
        size = ctypes.c_uint64()
        rc = self._lib.sz4_compress_blocks_device(self._h, ctypes.c_void_p(d_in), n, block_size, int(max_chain_length),
                                                  HEADERS[header], ctypes.c_void_p(d_out), out_cap,
                                                  ctypes.byref(size), ctypes.c_void_p(stream))
        self._check(rc, "sz4_compress_blocks_device")
        return size.value

    def compress_blocks(self, data, block_size: int = 65536, max_chain_length: int = MaxChainLength,
                        header: str = "smallz4") -> bytes:
        """Host bytes (or a uint8 torch tensor on the GPU) in, frame bytes out."""
        import torch
        if isinstance(data, torch.Tensor):
            t = data.contiguous().view(torch.uint8).reshape(-1)
            if not t.is_cuda:
                t = t.cuda(self.device)
        else:
            raw = bytes(data)
            t = torch.frombuffer(bytearray(raw), dtype=torch.uint8) if raw else torch.empty(0, dtype=torch.uint8)
            t = t.cuda(self.device)
        n = t.numel()
        cap = self._lib.sz4_bound(n, block_size)
        out = torch.empty(max(cap, 16), dtype=torch.uint8, device=t.device)
        stream = torch.cuda.current_stream(t.device).cuda_stream
        size = self.compress_blocks_device(t.data_ptr() if n else out.data_ptr(), n, out.data_ptr(), cap,
                                           block_size, max_chain_length, header, stream)
        return out[:size].cpu().numpy().tobytes()

    # -- decoder: the reference's smallz4cat -----------------------------------------------------
    def unlz4(self, frame: bytes, dictionary: bytes = b"") -> bytes:
        """smallz4cat's unlz4 (smallz4cat.c:112-360) on the GPU: the bytes `frame` decodes to.
        Raises NativeError for a frame the reference decoder rejects."""
        frame, dic = bytes(frame), bytes(dictionary)
        size = ctypes.c_uint64()
        rc = self._lib.sz4_unlz4(self._h, frame, len(frame), dic or None, len(dic), None, 0, ctypes.byref(size))
        if rc == _native.SZ4_OK:
            return b""
        if rc != _native.SZ4_E_CAPACITY:
            self._check(rc, "sz4_unlz4")
        out = ctypes.create_string_buffer(size.value)
        rc = self._lib.sz4_unlz4(self._h, frame, len(frame), dic or None, len(dic), out, size.value, ctypes.byref(size))
        self._check(rc, "sz4_unlz4")
        return out.raw[:size.value]

    def unlz4_stream(self, read_byte, write, dictionary: bytes = b"") -> None:
        """smallz4cat's unlz4_userPtr over callbacks (sz4_unlz4_stream): read_byte() -> int,
        write(bytes) -- called with 64 KiB pieces and the remainder, as the reference flushes."""
        err = []

        def get(_user):
            try:
                return read_byte()
            except BaseException as e:  # noqa: BLE001
                err.append(e)
                return 0

        def send(data, n, _user):
            try:
                write(ctypes.string_at(data, n) if n else b"")
            except BaseException as e:  # noqa: BLE001
                err.append(e)

        g, s = _native.GET_BYTE(get), _native.SEND_OUT(send)
        dic = bytes(dictionary)
        rc = self._lib.sz4_unlz4_stream(self._h, g, s, dic if dic else None, len(dic), None)
        if err:
            raise err[0]
        self._check(rc, "sz4_unlz4_stream")

    def unlz4_device(self, d_frame: int, n: int, d_out: int, out_cap: int, d_dict: int = 0, dict_len: int = 0,
                     stream: int = 0) -> int:
        """Device pointers in, decoded size out (see sz4_unlz4_device); raises when out_cap is too small."""
        size = ctypes.c_uint64()
        rc = self._lib.sz4_unlz4_device(self._h, ctypes.c_void_p(d_frame), n, ctypes.c_void_p(d_dict), dict_len,
                                        ctypes.c_void_p(d_out), out_cap, ctypes.byref(size), ctypes.c_void_p(stream))
        self._check(rc, "sz4_unlz4_device")
        return size.value

    def last_block_sizes(self, nblocks: int) -> list[int]:
        arr = (ctypes.c_uint32 * max(nblocks, 1))()
        k = self._lib.sz4_last_block_sizes(self._h, arr, nblocks)
        if k < 0:
            raise _native.NativeError("sz4_last_block_sizes failed")
        return list(arr[:k])

    def debug_stop_after(self, stage: int):
        self._lib.sz4_debug_stop_after(self._h, int(stage))

    def debug_matches(self, n: int):
        import numpy as np
        ln = np.zeros(n, dtype=np.uint32)
        ds = np.zeros(n, dtype=np.uint16)
        self._check(self._lib.sz4_debug_matches(self._h, ln.ctypes.data, ds.ctypes.data, n), "sz4_debug_matches")
        return ln, ds

    def device_bytes(self) -> int:
        """Device memory held by this context (scratch, staging, output buffers)."""
        return int(self._lib.sz4_device_bytes(self._h))

    def trim(self):
        """Release every device and pinned host buffer this context holds (sz4_trim)."""
        self._lib.sz4_trim(self._h)

    def set_device_limit(self, nbytes: int):
        """Bound this context's device memory (sz4_set_device_limit; 0 = no bound)."""
        self._lib.sz4_set_device_limit(self._h, int(nbytes))

    def released_buffers(self) -> int:
        """Buffers released so far under the device bound or memory pressure (sz4_released_buffers)."""
        return int(self._lib.sz4_released_buffers(self._h))

    def dict_rounds(self) -> int:
        """Dictionary mode: match-finder rounds of the last chunk (sz4_dict_rounds; 0xFFFFFFFF: the
        chunk fell back to the in-order replay)."""
        return int(self._lib.sz4_dict_rounds(self._h))

    def unlz4_resolve_passes(self) -> int:
        """Pointer-jumping passes of the last split-mode decode (0: decoded block by block)."""
        return int(self._lib.sz4_unlz4_resolve_passes(self._h))

    def unlz4_index_parallel(self) -> bool:
        """Whether the last decode's block index came from the parallel index (not the serial walk)."""
        return bool(self._lib.sz4_unlz4_index_parallel(self._h))

    def set_timing(self, on: bool):
        self._lib.sz4_set_timing(self._h, int(on))

    def last_stage_ms(self) -> dict:
        arr = (ctypes.c_float * len(STAGES))()
        self._lib.sz4_last_stage_ms(self._h, arr, len(STAGES))
        return dict(zip(STAGES, list(arr)))


_default = None


def _ctx() -> Compressor:
    global _default
    if _default is None:
        _default = Compressor()
    return _default


def lz4(data: bytes, max_chain_length: int = MaxChainLength, dictionary: bytes = b"",
        use_legacy_format: bool = False) -> bytes:
    """smallz4::lz4 (smallz4.h:47-64) on the GPU."""
    return _ctx().lz4(data, max_chain_length, dictionary, use_legacy_format)


def compress_blocks(data, block_size: int = 65536, max_chain_length: int = MaxChainLength,
                    header: str = "smallz4") -> bytes:
    return _ctx().compress_blocks(data, block_size, max_chain_length, header)


def unlz4(frame: bytes, dictionary: bytes = b"") -> bytes:
    """smallz4cat's decoder (smallz4cat.c:112-360) on the GPU."""
    return _ctx().unlz4(frame, dictionary)
