"""Device memory of a context: the batch API's scratch per piece byte, trimming,
the device bound that releases buffers kept from calls of another kind, the split decoder's fallback
to block-by-block decoding when its scratch does not fit, and the drop-in pool's cap.  Every result is
checked byte for byte: a bound changes where buffers live, never the output.  Run with -m gpu."""
import ctypes

import pytest

from oracle import pyoracle
from smallz4_amd import synth

pytestmark = pytest.mark.gpu

GiB = 1 << 30


def _fresh():
    import smallz4_amd
    return smallz4_amd.Compressor(device=0)


@pytest.mark.parametrize("bs,bound", [(65536, 40.0), (262144, 50.0)])
def test_batch_scratch_per_piece_byte(bs, bound):
    """sz4_compress_blocks_device's scratch is a fixed multiple of its piece size: the stage-local arrays
    (sort elements, parse choices, range minima, tokens, walk slots) share one region.  Round 4 held
    about 75 bytes per piece byte."""
    import torch
    comp = _fresh()
    try:
        piece = 64 << 20
        comp.set_batch_chunk(piece)
        data = synth.zeros_urandom_range(0, 2 * piece, seed=10) if bs == 262144 else synth.enwik8_like(2 * piece, seed=5)
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
        frame = comp.compress_blocks(t, bs, 65535)
        per = comp.device_bytes() / piece
        print(f"{bs // 1024} KiB blocks: {comp.device_bytes() / 2**20:.1f} MiB for {piece >> 20} MiB pieces = {per:.1f} B per piece byte")
        assert per <= bound
        # the output is unchanged: the first blocks against the oracle
        pos = 7
        for k in range(3):
            blk = pyoracle.oz_block(data[k * bs:(k + 1) * bs], 65535)
            assert frame[pos:pos + len(blk)] == blk, k
            pos += len(blk)
    finally:
        comp.close()


def test_trim_releases_everything_and_the_next_call_is_identical(compressor):
    data = synth.enwik8_like(3 << 20, seed=31)
    a = compressor.compress_blocks(data, 65536, 65535)
    s = compressor.lz4(data[:1 << 20])
    assert compressor.device_bytes() > 0
    compressor.trim()
    assert compressor.device_bytes() == 0
    # the same shape again: the plan is cached on the host, its device copy must be uploaded again
    assert compressor.compress_blocks(data, 65536, 65535) == a
    assert compressor.lz4(data[:1 << 20]) == s
    assert compressor.unlz4(a) == data


def test_device_limit_releases_buffers_of_other_calls():
    """Stream compression (two chunk slots), dictionary mode and the decoder's split image leave buffers
    in the context; a batch call under a bound releases them instead of growing past it."""
    import torch
    comp = _fresh()
    try:
        comp.set_stream_chunk(8 << 20)
        text = synth.enwik8_like(24 << 20, seed=32)
        t = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
        free = comp.compress_blocks(t, 65536, 65535)
        need = comp.device_bytes()  # the batch call's own working set
        comp.trim()
        st = comp.lz4(text)
        d = comp.lz4(text[:2 << 20], dictionary=text[-70000:])
        assert comp.unlz4(st) == text
        held = comp.device_bytes()
        before = comp.released_buffers()
        limit = int(need * 1.15)
        assert limit < held + need
        comp.set_device_limit(limit)
        assert comp.compress_blocks(t, 65536, 65535) == free
        assert comp.device_bytes() <= limit
        assert comp.released_buffers() > before
        # the released kinds still work (they allocate again, under the same bound when they fit)
        comp.set_device_limit(0)
        assert comp.lz4(text[:2 << 20], dictionary=text[-70000:]) == d
    finally:
        comp.close()


def test_split_decoder_falls_back_to_blockwise_under_limit():
    """split-mode decoding (blocks of >= 256 KiB payload) needs about twice the per-block
    decoder's scratch; when it does not fit the frame decodes block by block instead of failing."""
    comp = _fresh()
    try:
        text = synth.enwik8_like(24 << 20, seed=33)
        frame = comp.lz4(text)  # 4 MiB dependent blocks: split mode
        comp.trim()
        assert comp.unlz4(frame) == text
        split_bytes = comp.device_bytes()
        comp.trim()
        # per-block mode: frame + output + ~5.3 x frame of sequence lists; split mode: ~10.7 x frame + 4 x output
        limit = len(frame) * 8 + len(text) * 2
        assert limit < split_bytes, (limit, split_bytes)
        comp.set_device_limit(limit)
        assert comp.unlz4(frame) == text
        assert comp.device_bytes() <= limit
        comp.set_device_limit(len(text) // 2)  # not even the output fits: a clean error, no crash
        comp.trim()
        with pytest.raises(Exception):
            comp.unlz4(frame)
        comp.set_device_limit(0)
        assert comp.unlz4(frame) == text
    finally:
        comp.close()


def test_split_decoder_output_counted_under_limit():
    """a bound between the split plan's own buffers and those plus the output buffer.  The
    split plan fits, the output does not beside it: the frame is planned again block by block (and the
    index scratch is released) instead of failing with SZ4_E_NOMEM."""
    comp = _fresh()
    try:
        text = synth.enwik8_like(24 << 20, seed=36)
        frame = comp.lz4(text)  # 4 MiB dependent blocks: split mode
        comp.trim()
        assert comp.unlz4(frame) == text
        whole = comp.device_bytes()  # frame + split plan + index scratch + output
        comp.trim()
        limit = whole - len(text) // 2  # the plan fits, the output beside it does not
        comp.set_device_limit(limit)
        assert comp.unlz4(frame) == text
        assert comp.device_bytes() <= limit
        comp.set_device_limit(0)
    finally:
        comp.close()


def test_pool_cap_trims_released_contexts():
    """The drop-in's context pool: a context returned holding more than the cap is trimmed."""
    from smallz4_amd import _native
    lib = _native.lib()
    data = synth.enwik8_like(6 << 20, seed=34)
    out = ctypes.create_string_buffer(lib.sz4_lz4_bound(len(data), 0))
    size = ctypes.c_uint64(0)
    h = ctypes.c_void_p()
    try:
        lib.sz4_set_pool_cap(1 << 20)
        assert lib.sz4_acquire(ctypes.byref(h), 0) == 0
        assert lib.sz4_lz4(h, data, len(data), 65535, None, 0, 0, out, len(out), ctypes.byref(size)) == 0
        frame = out.raw[:size.value]
        assert lib.sz4_device_bytes(h) > (1 << 20)
        lib.sz4_release(h)
        assert lib.sz4_device_bytes(h) == 0
        h2 = ctypes.c_void_p()
        assert lib.sz4_acquire(ctypes.byref(h2), 0) == 0
        assert lib.sz4_lz4(h2, data, len(data), 65535, None, 0, 0, out, len(out), ctypes.byref(size)) == 0
        assert out.raw[:size.value] == frame
        lib.sz4_release(h2)
    finally:
        lib.sz4_set_pool_cap(0)


def test_batch_4gib_shared_context_after_stream_and_dictionary(compressor):
    """4 GiB of configs[4]'s shape in one call on the SHARED session context, after
    it has served stream, dictionary and decoder calls, under a 24 GiB bound.  Round 4 needed a context
    of its own (the shared one reached 24.01 GiB)."""
    import test_shards
    text = synth.enwik8_like(140 << 20, seed=35)
    assert compressor.unlz4(compressor.lz4(text)) == text  # two 64 MiB chunk slots, split decoder
    compressor.lz4(text[:3 << 20], dictionary=text[-65536:])
    del text
    compressor.set_device_limit(24 * GiB)
    try:
        test_shards._batch_4gib(compressor, __import__("torch"))
        print(f"released {compressor.released_buffers()} buffers kept from the stream/dictionary/decoder calls")
    finally:
        compressor.set_device_limit(0)
