"""The bounded-memory stream paths (sz4_lz4_stream / sz4_lz4 compressing chunk by chunk, and
sz4_unlz4_stream decoding chunk by chunk) against the reference's golden vectors and the oracle.
A chunk boundary must not change a byte: the carried 64 KiB window, the lookback cut and the previous
block's shortcut intervals (smallz4.h:614-643, 798-805) and dictionary mode's tables all cross it.
Also: reentrancy of the drop-in header (threads), and a multi-GiB stream with a fixed device
footprint.  Run with -m gpu on an MI355X."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

import inputs
from oracle import pyoracle
from smallz4_amd import synth

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M = 4 << 20  # MaxBlockSize


@pytest.fixture
def chunked(compressor):
    """The compressor with one 4 MiB block per chunk: every block boundary is a chunk boundary."""
    compressor.set_stream_chunk(M)
    yield compressor
    compressor.set_stream_chunk(0)


def test_golden_vectors_one_block_per_chunk(chunked, golden):
    for case in golden:
        data = inputs.make(case["input"])
        dictionary = inputs.make(case["dict"]) if "dict" in case else b""
        frame = chunked.lz4(data, case["level"], dictionary, bool(case["legacy"]))
        assert inputs.sha(frame) == case["out_sha256"], (case["name"], case["level"], case["legacy"])


CASES = {
    "text9m": lambda: synth.enwik8_like(9 << 20, seed=60),
    # a zero run of 110 000 bytes across the first block boundary: the same-letter shortcut interval
    # of block 0 reaches its end, so block 1's window must leave those positions out (the ghost slot)
    "run_across": lambda: synth.enwik8_like(M - 40000, seed=61) + bytes(110000) + synth.enwik8_like(M + 70000, seed=62),
    "edge": lambda: synth.enwik8_like(M - 20, seed=63) + bytes(100) + synth.enwik8_like(M + 5, seed=64),
}


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("chain", [2, 5, 7, 65535])
def test_chunk_boundaries_match_oracle(chunked, chain, case):
    data = CASES[case]()
    assert chunked.lz4(data, chain) == pyoracle.oz_lz4(data, chain)


@pytest.mark.parametrize("chain", [5, 65535])
def test_multi_block_chunks_carry_state(compressor, chain):
    """Chunks of two and three 4 MiB blocks: the ghost slot then carries the intervals of a chunk's
    LAST block (B.prev = nb) across the boundary; a zero run crosses the first chunk boundary and
    another lies inside a chunk.  The whole frame against the oracle."""
    # the reference's frame (tests/golden/streams.json, carry_state_l*: its walk is quadratic in the runs)
    case, data, _ = _stream_case(f"carry_state_l{chain}")
    assert data == (synth.enwik8_like(2 * M - 50000, seed=92) + bytes(120000) + synth.enwik8_like(M, seed=93) +
                    bytes(90000) + synth.enwik8_like(2 * M + 12345, seed=94))
    for chunk in (2 * M, 3 * M):
        compressor.set_stream_chunk(chunk)
        try:
            out = compressor.lz4(data, chain)
            assert len(out) == case["frame_len"] and inputs.sha(out) == case["frame_sha256"], chunk
        finally:
            compressor.set_stream_chunk(0)


def test_stream_rejects_oversized_reads(compressor):
    """A read callback that returns more bytes than it was asked for is an error, not an overrun."""
    data = synth.enwik8_like(300000, seed=95)
    with pytest.raises(ValueError):
        compressor.lz4_stream(lambda n: data, lambda b: None, 65535)


def test_decoder_stream_rejects_huge_block_word(compressor):
    """A size word larger than any LZ4 block is corrupt (checked before anything is reserved)."""
    from smallz4_amd._native import NativeError
    frame = bytes([0x04, 0x22, 0x4D, 0x18, 0x40, 0x70, 0xDF]) + (0x7FFFFFF0).to_bytes(4, "little") + bytes(64)
    with pytest.raises(NativeError, match="larger than any LZ4 block"):
        _decode_stream(compressor, frame)


@pytest.mark.parametrize("legacy,chain", [(False, 3), (False, 6), (False, 65535), (True, 3), (True, 6)])
def test_chunked_dictionary(chunked, chain, legacy):
    """Dictionary mode carries the reference's hash table and both chains across chunks (their slots
    are absolute positions mod 65536: chunks move by multiples of 65536).  Modern frames take the
    data-parallel path (sz4_dict.hip), legacy frames replay the reference's loop in one wavefront
    (DESIGN.md section 3.7), so those run at short chains only."""
    data = synth.enwik8_like(2 * M + 300000, seed=66)
    dictionary = synth.enwik8_like(50000, seed=67)
    assert chunked.lz4(data, chain, dictionary, legacy) == pyoracle.oz_lz4(data, chain, dictionary, legacy)


@pytest.mark.parametrize("chain", [3, 65535])
def test_chunked_dictionary_multi_block_chunks(compressor, chain):
    """Chunks of two 4 MiB blocks with a dictionary: the snapshot reads of the chain slots cross a block
    boundary inside a chunk and the carried tables cross the chunk boundary."""
    data = synth.enwik8_like(4 * M + 123457, seed=68)
    dictionary = synth.enwik8_like(65536, seed=69)
    compressor.set_stream_chunk(2 * M)
    try:
        assert compressor.lz4(data, chain, dictionary) == pyoracle.oz_lz4(data, chain, dictionary)
    finally:
        compressor.set_stream_chunk(0)


@pytest.mark.parametrize("chain", [3, 6])
def test_dictionary_long_run_rounds(chunked, chain):
    """A run of one byte value long enough for the same-letter shortcut (> 65 300 bytes) in dictionary
    mode: the data-parallel finder runs its chunk again with the shortcut intervals its first results
    imply (sz4_dict.hip), and the next chunk continues from the tables that round left.  No in-order
    replay."""
    data = (synth.enwik8_like(M - 120000, seed=70) + b"a" * 70000 + synth.enwik8_like(50000, seed=71) +
            bytes(30000) + synth.enwik8_like(M // 2, seed=72))
    dictionary = b"a" * 1000 + synth.enwik8_like(9000, seed=73)
    assert chunked.lz4(data, chain, dictionary) == pyoracle.oz_lz4(data, chain, dictionary)
    assert chunked.dict_rounds() != 0xFFFFFFFF


def _streams_golden():
    with open(os.path.join(ROOT, "tests", "golden", "streams.json")) as f:
        return {c["name"]: c for c in json.load(f)["cases"]}


def _stream_case(name):
    case = _streams_golden()[name]
    data = inputs.make(case["input"])
    assert inputs.sha(data) == case["input_sha256"]
    dic = inputs.make(case["dictionary"]) if case["dictionary"] else b""
    assert inputs.sha(dic) == case["dictionary_sha256"]
    return case, data, dic


@pytest.mark.parametrize("name", sorted(n for n in _streams_golden() if n.startswith("dict_")))
def test_dictionary_stream_fixtures(compressor, name):
    """The reference's own frames for dictionary streams it is too slow to redo inside a test
    (tests/golden/streams.json, made by make_streams_golden.py: a long run makes its chain walk
    quadratic): runs long enough for the same-letter shortcut -- in the middle of 8 MB, across blocks,
    at a 16 KiB-unaligned offset, in configs[4]-shaped zeros/urandom data -- and legacy frames with a
    dictionary, at -9, -6 and -3.  All on the data-parallel path (no in-order replay)."""
    case, data, dic = _stream_case(name)
    out = compressor.lz4(data, case["max_chain"], dic, case["legacy"])
    assert len(out) == case["frame_len"] and inputs.sha(out) == case["frame_sha256"]
    assert compressor.dict_rounds() != 0xFFFFFFFF


@pytest.mark.parametrize("name", ["dict_zero_run_8m_l9", "dict_legacy_12m_l9"])
def test_dictionary_throughput_floor(compressor, name):
    """Dictionary mode has no serial cliff: 8 MB with a 64 KiB dictionary and a 200 KB zero run (the
    same-letter shortcut) and a 12 MB legacy frame with a dictionary both compress at >= 100 MB/s at -9,
    byte-identical to the reference (host buffers in and out, the second call timed)."""
    import time
    case, data, dic = _stream_case(name)
    compressor.lz4(data[:1 << 20], case["max_chain"], dic, case["legacy"])
    # the best of three calls (one timed call on a shared box is a flaky gate); the byte
    # identity is checked on every call
    rate = 0.0
    for _ in range(3):
        t0 = time.perf_counter()
        out = compressor.lz4(data, case["max_chain"], dic, case["legacy"])
        rate = max(rate, len(data) / (time.perf_counter() - t0) / 1e6)
        assert inputs.sha(out) == case["frame_sha256"]
    print(f"{name}: {rate:.1f} MB/s, {compressor.dict_rounds()} rounds")
    assert rate >= 100.0, rate


def test_dictionary_replay_fallback(monkeypatch):
    """the in-order replay that takes a dictionary chunk whose shortcut rounds do not settle
    (k_dict_matches, after the saved tables are restored) forced on a context created with
    SZ4_DICT_NO_GUESS=1 (the first round assumes no interval, so a long run needs a second round) and
    SZ4_DICT_MAX_ROUNDS=1: the same bytes as the oracle, and the fallback reported across the call's
    chunks (a first chunk that falls back, a second that does not)."""
    import smallz4_amd
    monkeypatch.setenv("SZ4_DICT_NO_GUESS", "1")
    monkeypatch.setenv("SZ4_DICT_MAX_ROUNDS", "1")
    comp = smallz4_amd.Compressor(device=0)
    try:
        comp.set_stream_chunk(M)
        data = (synth.enwik8_like(200000, seed=74) + b"q" * 70000 + synth.enwik8_like(M - 270000 + 5000, seed=75) +
                synth.enwik8_like(300000, seed=76))
        dictionary = synth.enwik8_like(40000, seed=77)
        for chain in (3, 6):
            assert comp.lz4(data, chain, dictionary) == pyoracle.oz_lz4(data, chain, dictionary)
            assert comp.dict_rounds() == 0xFFFFFFFF, chain
    finally:
        comp.close()


@pytest.mark.parametrize("chain", [3, 6])
def test_dictionary_rounds_bounded_many_runs(compressor, chain):
    """many same-letter runs in one block at greedy/lazy levels settle in a few rounds (the
    run-table guess), far below the cap that hands a chunk to the in-order replay."""
    parts = []
    for k in range(24):
        parts.append(synth.enwik8_like(9000 + 37 * k, seed=80 + k))
        parts.append(bytes([65 + k]) * (65400 + 211 * k))
    data = b"".join(parts)
    dictionary = synth.enwik8_like(65536, seed=79)
    assert compressor.lz4(data, chain, dictionary) == pyoracle.oz_lz4(data, chain, dictionary)
    rounds = compressor.dict_rounds()
    print(f"{len(data)} bytes, 24 runs: {rounds} rounds")
    assert 1 <= rounds <= 4, rounds


@pytest.mark.parametrize("chain", [3, 65535])
def test_chunked_legacy(chunked, chain):
    data = synth.enwik8_like(2 * (8 << 20) + 300000, seed=66)
    assert chunked.lz4(data, chain, b"", True) == pyoracle.oz_lz4(data, chain, b"", True)


def test_stream_callbacks_ragged_reads(chunked):
    """getBytes may return fewer bytes than asked; the output and the call pattern stay the reference's."""
    data = synth.enwik8_like(2 * M + 777, seed=68)
    rng = np.random.default_rng(69)
    pos = [0]

    def read(n):
        k = int(min(n, rng.integers(1, 70000), len(data) - pos[0]))
        b = data[pos[0]:pos[0] + k]
        pos[0] += k
        return b

    calls = []
    chunked.lz4_stream(read, calls.append, 65535)
    want = pyoracle.oz_lz4(data, 65535)
    assert b"".join(calls) == want
    # header, then per block 4 one-byte calls and the payload, then the end mark (smallz4.h:478-812)
    nblocks = (len(data) + M - 1) // M
    assert len(calls) == 1 + 5 * nblocks + 1
    assert calls[0] == want[:7] and all(len(c) == 1 for c in calls[1:5]) and calls[-1] == b"\0\0\0\0"


def test_stream_empty_and_tiny(compressor):
    for data in (b"", b"a", b"abcdefghijkl"):
        for legacy in (False, True):
            out = []
            compressor.lz4_stream(lambda n, d=[data]: d.pop() if d else b"", out.append, 65535, b"", legacy)
            assert b"".join(out) == pyoracle.oz_lz4(data, 65535, b"", legacy)


def _decode_stream(compressor, frame, dictionary=b""):
    it = iter(frame)
    pieces = []
    compressor.unlz4_stream(lambda: next(it), pieces.append, dictionary)
    return pieces


@pytest.mark.parametrize("legacy", [False, True])
def test_decoder_stream_chunks_and_flush_points(compressor, legacy):
    compressor.set_stream_chunk(2 << 20)  # 1 MiB of frame per decode chunk
    try:
        data = synth.enwik8_like(3 * M + 1000, seed=70)
        frame = pyoracle.oz_lz4(data, 65535, b"", legacy)
        pieces = _decode_stream(compressor, frame)
        assert b"".join(pieces) == data
        # the reference flushes its 64 KiB history whenever it fills, and the remainder at the end
        assert all(len(p) == 65536 for p in pieces[:-1]) and len(pieces[-1]) == len(data) % 65536
        dictionary = synth.enwik8_like(90000, seed=71)
        frame = pyoracle.oz_lz4(data[:300000], 6, dictionary, legacy)
        assert b"".join(_decode_stream(compressor, frame, dictionary)) == pyoracle.oz_unlz4(frame, dictionary)
    finally:
        compressor.set_stream_chunk(0)


def test_decoder_stream_rejects_like_the_reference(compressor):
    from smallz4_amd._native import NativeError
    with pytest.raises(NativeError, match="invalid signature"):
        _decode_stream(compressor, b"\x00\x01\x02\x03" + bytes(20))
    with pytest.raises(NativeError, match="version 1"):
        _decode_stream(compressor, bytes([0x04, 0x22, 0x4D, 0x18, 0x80, 0x70, 0xDF]) + bytes(8))


def _build_tool(tmp_path):
    exe = tmp_path / "stream_threads"
    subprocess.run(["hipcc", "-std=c++17", "-O2", "-pthread", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "stream_threads.cpp"), "-L", os.path.join(ROOT, "smallz4_amd", "lib"),
                    "-lsmallz4_amd", "-Wl,-rpath," + os.path.join(ROOT, "smallz4_amd", "lib"), "-o", str(exe)], check=True)
    return str(exe)


def test_dropin_concurrent_threads(tmp_path):
    """Four host threads call smallz4::lz4 at once (include/smallz4_amd.hpp): each gets a context of
    its own from the library's pool, and each output equals the oracle's."""
    exe = _build_tool(tmp_path)
    datas = [synth.enwik8_like((1 << 20) * (k + 1) + 333 * k, seed=80 + k) for k in range(4)]
    args = [exe, "threads", "9"]
    for k, d in enumerate(datas):
        (tmp_path / f"in{k}").write_bytes(d)
        args += [str(tmp_path / f"in{k}"), str(tmp_path / f"out{k}")]
    subprocess.run(args, check=True, timeout=300)
    for k, d in enumerate(datas):
        assert (tmp_path / f"out{k}").read_bytes() == pyoracle.oz_lz4(d, 65535), k


def _big_input(base: bytes, reps: int) -> bytes:
    buf = bytearray(base * reps)
    size = len(base)
    for r in range(reps):
        p = (r * 7919) % size
        for j in range(8):
            if p + j < size:
                buf[r * size + p + j] = (r >> (8 * j)) & 0xFF
    return bytes(buf)


def test_dropin_multi_gib_stream_fixed_footprint(tmp_path):
    """2 GiB through smallz4::lz4 in 64 MiB chunks: the device footprint is that of one chunk, the
    frame decodes to the input (oracle decoder), and its first blocks equal the oracle's stream."""
    exe = _build_tool(tmp_path)
    base = synth.enwik8_like(16 << 20, seed=90)
    (tmp_path / "base").write_bytes(base)
    reps = 128
    r = subprocess.run([exe, "big", "9", str(tmp_path / "base"), str(reps), str(tmp_path / "big.lz4")],
                       check=True, capture_output=True, text=True, timeout=600)
    info = json.loads(r.stdout.strip().splitlines()[-1])
    assert info["input_bytes"] == reps * len(base)
    assert info["device_bytes"] < 8 << 30, info  # one 64 MiB chunk's scratch, not 2 GiB worth
    frame = (tmp_path / "big.lz4").read_bytes()
    assert len(frame) == info["output_bytes"]
    data = _big_input(base, reps)
    assert hashlib.sha256(pyoracle.oz_unlz4(frame, cap=len(data) + 16)).digest() == hashlib.sha256(data).digest()
    head = pyoracle.oz_lz4(data[:3 * M], 65535)
    assert frame[:len(head) - 4] == head[:-4]
