"""The device decoder (sz4_unlz4 / sz4_unlz4_device: the reference's smallz4cat,
smallz4cat.c:112-360) against the oracle's restatement of it (oz_unlz4, pinned against the
reference's own smallz4cat binary in tests/test_oracle.py) and, where that binary was compiled
(oracle/_ref/smallz4cat), against the reference itself.  Byte-for-byte; a frame the oracle rejects
must raise.  Run with -m gpu on an MI355X."""
import os
import struct
import subprocess

import numpy as np
import pytest

import inputs
from oracle import pyoracle
from smallz4_amd import synth
from smallz4_amd._native import NativeError

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAGIC = bytes([0x04, 0x22, 0x4D, 0x18])


def oracle_decode(frame, dictionary=b""):
    """oz_unlz4's output, or None when it rejects the frame."""
    try:
        return pyoracle.oz_unlz4(frame, dictionary, cap=(1 << 20) + 300 * len(frame))
    except ValueError:
        return None


def check(compressor, frame, dictionary=b""):
    want = oracle_decode(frame, dictionary)
    if want is None:
        with pytest.raises(NativeError):
            compressor.unlz4(frame, dictionary)
    else:
        assert compressor.unlz4(frame, dictionary) == want
    return want


def blocks_of(frame):
    """(word, payload) of every block of a modern frame with the 7-byte smallz4 header."""
    pos, out = 7, []
    while True:
        word = int.from_bytes(frame[pos:pos + 4], "little")
        pos += 4
        if word == 0:
            return out
        n = word & 0x7FFFFFFF
        out.append((word, frame[pos:pos + n]))
        pos += n


def build_frame(flags, blocks, content=0, tail=b""):
    """A modern frame with descriptor FLG `flags`: optional content size, dictionary ID, block and
    content checksums (arbitrary bytes: the reference skips them, smallz4cat.c:129-159, 345-356)."""
    hdr = MAGIC + bytes([flags, 0x70])
    if flags & 8:
        hdr += struct.pack("<Q", content)
    if flags & 1:
        hdr += b"\x11\x22\x33\x44"
    hdr += b"\xAB"
    body = b""
    for word, payload in blocks:
        body += struct.pack("<I", word) + payload
        if flags & 16:
            body += b"\xDE\xAD\xBE\xEF"
    return hdr + body + b"\0\0\0\0" + (b"\x01\x02\x03\x04" if flags & 4 else b"") + tail


def test_unlz4_golden_streams(compressor, golden):
    """Every golden vector's frame (the reference's bytes, regenerated on the GPU and checked against
    the vector's SHA-256) decodes as the oracle decodes it: to the input, except the dictionary frames
    the reference itself cannot decode, where both give the same bytes."""
    for case in golden:
        data = inputs.make(case["input"])
        dictionary = inputs.make(case["dict"]) if "dict" in case else b""
        frame = compressor.lz4(data, case["level"], dictionary, bool(case["legacy"]))
        assert inputs.sha(frame) == case["out_sha256"]
        got = check(compressor, frame, dictionary)
        if case["legacy"] and case["level"] == 0:
            # the reference writes an empty block for a legacy frame at level 0, and its smallz4cat
            # decodes that to nothing (a reference defect, reproduced: tests/test_oracle.py)
            assert got == b"", case["name"]
        elif not dictionary:
            assert got == data, (case["name"], case["level"], case["legacy"])


@pytest.mark.parametrize("bs", [1000, 65536, 1 << 20, 4 << 20])
@pytest.mark.parametrize("chain", [0, 3, 65535])
def test_unlz4_independent_blocks(compressor, bs, chain):
    data = synth.enwik8_like(3 << 20, seed=60) + synth.random_bytes(300000, seed=61) + bytes(200000)
    frame = compressor.compress_blocks(data, bs, chain)
    assert check(compressor, frame) == data


@pytest.mark.parametrize("legacy", [False, True])
def test_unlz4_dependent_stream(compressor, legacy):
    """4 MiB blocks that reference the block before them (a wait on its done flag); legacy 8 MiB
    blocks, including a last block of exactly 8 MiB (the frame ends at the end of the input)."""
    data = synth.enwik8_like(9 << 20, seed=62)
    assert check(compressor, compressor.lz4(data, 65535, b"", legacy)) == data
    if legacy:
        d8 = data[:8 << 20]
        assert check(compressor, compressor.lz4(d8, 6, b"", True)) == d8


def test_unlz4_frame_descriptor_fields(compressor):
    data = synth.enwik8_like(300000, seed=63)
    blocks = blocks_of(compressor.compress_blocks(data, 65536, 65535))
    for flags in (0x40, 0x50, 0x48, 0x44, 0x41, 0x5D, 0x60, 0x7D):
        assert check(compressor, build_frame(flags, blocks, content=len(data))) == data, hex(flags)
    assert check(compressor, build_frame(0x40, blocks, tail=b"trailing bytes")) == data


def test_unlz4_malformed(compressor):
    """Frames the reference decoder rejects raise (the oracle says which)."""
    data = synth.enwik8_like(70000, seed=64)
    good = compressor.compress_blocks(data, 65536, 65535)
    hdr = MAGIC + b"\x40\x70\xdf"
    cases = [b"", b"\x04\x22", b"\x00\x22\x4d\x18\x40\x70\xdf\0\0\0\0",
             MAGIC + b"\x00\x70\xdf\0\0\0\0",                               # version 0
             hdr + b"\x04\0\0\0" + b"\x10a\x00\x00" + b"\0\0\0\0",          # offset 0
             hdr + b"\x03\0\0\0" + b"\xF0\xFF\x05" + b"\0\0\0\0",           # literal run past its block
             hdr + b"\x02\0\0\0" + b"\x1Fa" + b"\0\0\0\0"]                  # offset past its block
    cases += [good[:k] for k in range(0, len(good), max(1, len(good) // 97))]
    for frame in cases:
        check(compressor, frame)


def test_unlz4_fuzz(compressor):
    """Random byte changes of small frames: the device returns what the oracle returns, or raises
    where the oracle rejects."""
    rng = np.random.default_rng(65)
    base = [compressor.compress_blocks(synth.enwik8_like(5000, seed=66), 1024, 65535),
            compressor.lz4(synth.runs(6000, seed=67, max_run=300), 65535)]
    for i in range(300):
        f = bytearray(base[i % 2])
        for _ in range(int(rng.integers(1, 4))):
            k = int(rng.integers(7, len(f)))
            f[k] = int(rng.integers(0, 256))
        check(compressor, bytes(f))


def test_unlz4_dictionary(compressor):
    """The dictionary's last 64 KiB precede the output (smallz4cat.c:168-187); references before
    it read the oracle's zero history."""
    data = synth.enwik8_like(50000, seed=68)
    for dictionary in (synth.enwik8_like(20000, seed=69), synth.enwik8_like(90000, seed=70), b"tiny"):
        for legacy in (False, True):
            check(compressor, compressor.lz4(data, 65535, dictionary, legacy), dictionary)
    # 4 literals, a match 10 back (6 into the dictionary, overlapping its own output), a match
    # 40000 back (before a short dictionary: zeros), one closing literal
    payload = b"\x44abcd\x0a\x00" + b"\x01\x40\x9c" + b"\x10z"
    frame = MAGIC + b"\x40\x70\xdf" + struct.pack("<I", len(payload)) + payload + b"\0\0\0\0"
    for d in (b"0123456789", b"", synth.random_bytes(70000, seed=71)):
        got = check(compressor, frame, d)
        assert got is not None and len(got) == 18


def test_unlz4_device_api_roundtrip_100mb(compressor):
    """100 MB in HBM: compressed (64 KiB blocks, -9) and decoded on the device, equal to the input."""
    import torch
    data = synth.enwik8_like(100_000_000, seed=72)
    t = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    frame = compressor.compress_blocks(t, 65536, 65535)
    f = torch.frombuffer(bytearray(frame), dtype=torch.uint8).cuda()
    out = torch.empty(len(data), dtype=torch.uint8, device="cuda")
    n = compressor.unlz4_device(f.data_ptr(), len(frame), out.data_ptr(), len(data))
    assert n == len(data) and torch.equal(out, t)
    assert compressor.unlz4_index_parallel()  # 1526 blocks indexed without the serial walk
    with pytest.raises(NativeError):
        compressor.unlz4_device(f.data_ptr(), len(frame), out.data_ptr(), len(data) - 1)


@pytest.mark.skipif(not os.path.exists(pyoracle.REF_CAT), reason="reference decoder not compiled")
def test_unlz4_matches_reference_binary(compressor, tmp_path):
    """The reference's own smallz4cat (built from /root/reference by oracle/Makefile) writes the same
    bytes: modern, legacy, stored, descriptor fields, a dictionary of >= 64 KiB."""
    data = synth.enwik8_like(2 << 20, seed=73) + synth.random_bytes(100000, seed=74)
    dic = synth.enwik8_like(70000, seed=75)
    dpath = tmp_path / "dict.bin"
    dpath.write_bytes(dic)
    frames = [(compressor.lz4(data, 65535), None), (compressor.lz4(data, 0), None),
              (compressor.lz4(data, 6, b"", True), None),
              (build_frame(0x5D, blocks_of(compressor.compress_blocks(data, 65536, 9)), content=len(data)), None),
              (compressor.lz4(data[:200000], 65535, dic), dpath)]
    for frame, d in frames:
        args = [pyoracle.REF_CAT] + (["-D", str(d)] if d else [])
        ref = subprocess.run(args, input=frame, capture_output=True, check=True).stdout
        assert compressor.unlz4(frame, dic if d else b"") == ref


def test_unlz4_c_dropin_program(compressor, tmp_path):
    """tests/cpp/unlz4_demo.c -- smallz4cat's main over include/smallz4cat_amd.h -- decodes stdin."""
    exe = tmp_path / "unlz4_demo"
    lib = os.path.join(ROOT, "smallz4_amd", "lib")
    subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "unlz4_demo.c"), "-L", lib, "-lsmallz4_amd",
                    "-Wl,-rpath," + lib, "-Wl,--allow-shlib-undefined", "-o", str(exe)], check=True)
    data = synth.enwik8_like(5 << 20, seed=76)
    for legacy in (False, True):
        r = subprocess.run([str(exe)], input=compressor.lz4(data, 6, b"", legacy), capture_output=True, check=True)
        assert r.stdout == data
    dic = tmp_path / "dict.bin"
    dic.write_bytes(synth.enwik8_like(80000, seed=77))
    frame = compressor.lz4(data[:100000], 65535, dic.read_bytes())
    r = subprocess.run([str(exe), "-D", str(dic)], input=frame, capture_output=True, check=True)
    assert r.stdout == pyoracle.oz_unlz4(frame, dic.read_bytes())
    bad = subprocess.run([str(exe)], input=b"not a frame", capture_output=True)
    assert bad.returncode == 1 and bad.stderr.startswith(b"ERROR: ")


@pytest.fixture(scope="module")
def split():
    """A context whose decoder runs every frame in split mode (SZ4_UNLZ4_SPLIT=1): blocks cut into
    8 KiB sub-segments parsed speculatively and joined to the true token chain (k_unlz4_spec /
    k_unlz4_fix), decoded one wavefront per sub-segment into a value-or-reference image whose references
    are resolved by pointer jumping (k_unlz4_sub / k_unlz4_resolve / k_unlz4_pack)."""
    import smallz4_amd
    os.environ["SZ4_UNLZ4_SPLIT"] = "1"
    try:
        c = smallz4_amd.Compressor(device=0)
    finally:
        del os.environ["SZ4_UNLZ4_SPLIT"]
    yield c
    c.close()


def test_unlz4_split_mode_matches_oracle(compressor, split, golden):
    """Split mode gives the oracle's bytes (or rejects where it rejects) on every frame shape: the golden
    vectors' frames, independent blocks from 1000 B to 4 MiB at levels 0 / 3 / 9 (stored blocks
    included), dependent 4 MiB and legacy 8 MiB streams, dictionaries, malformed and mutated frames."""
    for case in golden:
        data = inputs.make(case["input"])
        dictionary = inputs.make(case["dict"]) if "dict" in case else b""
        check(split, compressor.lz4(data, case["level"], dictionary, bool(case["legacy"])), dictionary)
    data = synth.enwik8_like(3 << 20, seed=60) + synth.random_bytes(300000, seed=61) + bytes(200000)
    for bs in (1000, 65536, 1 << 20, 4 << 20):
        for chain in (0, 3, 65535):
            assert check(split, compressor.compress_blocks(data, bs, chain)) == data, (bs, chain)
    d9 = synth.enwik8_like(9 << 20, seed=62) + bytes(3 << 20) + synth.runs(2 << 20, seed=72, max_run=70000)
    for legacy in (False, True):
        assert check(split, compressor.lz4(d9, 65535, b"", legacy)) == d9, legacy
    small = synth.enwik8_like(50000, seed=68)
    for dictionary in (synth.enwik8_like(20000, seed=69), synth.enwik8_like(90000, seed=70), b"tiny"):
        check(split, compressor.lz4(small, 65535, dictionary), dictionary)
    good = compressor.compress_blocks(synth.enwik8_like(70000, seed=64), 65536, 65535)
    for frame in [good[:k] for k in range(0, len(good), max(1, len(good) // 53))]:
        check(split, frame)
    rng = np.random.default_rng(73)
    base = compressor.lz4(synth.runs(20000, seed=67, max_run=300), 65535)
    for _ in range(150):
        f = bytearray(base)
        for _ in range(int(rng.integers(1, 4))):
            k = int(rng.integers(7, len(f)))
            f[k] = int(rng.integers(0, 256))
        check(split, bytes(f))


def test_unlz4_split_mode_large_roundtrip(compressor):
    """The automatic choice: a stream of 4 MiB dependent blocks (smallz4::lz4) takes split mode and
    decodes back on the device, text plus long runs."""
    data = synth.silesia_like(24 << 20, seed=74)
    frame = compressor.lz4(data, 65535)
    assert compressor.unlz4(frame) == data


def test_unlz4_index_false_candidates(compressor):
    """The parallel frame index (sz4_unlz4.hip, k_unlz4_ix_*) takes every offset whose size-word chain
    stays inside the frame for three hops as a candidate.  Stored blocks whose payload is itself an LZ4
    frame of 1000-byte blocks hold thousands of such chains (and zero words: end marks) next to the true
    one; the walk from the first size word must step over them.  Modern and legacy outer frames."""
    text = synth.enwik8_like(400000, seed=74)
    inner = compressor.compress_blocks(text, 1000, 65535)
    inner_legacy = compressor.lz4(text, 65535, b"", True)
    payload = synth.random_bytes(70001, seed=75) + inner + bytes(5) + inner_legacy + inner
    # (legacy frames at level 1: the reference writes a legacy frame at level 0 with an empty block, see
    # test_unlz4_golden_streams; its literals still carry the inner frames' size words)
    for frame in (compressor.compress_blocks(payload, 65536, 0), compressor.compress_blocks(payload, 4099, 0),
                  compressor.lz4(payload, 1, b"", True), compressor.lz4(payload, 0)):
        assert check(compressor, frame) == payload
        assert compressor.unlz4_index_parallel()
    # truncated and bit-flipped outer frames: the index decides exactly as the one-lane walk
    frame = compressor.compress_blocks(payload, 65536, 0)
    for k in (7, 11, 65540 + 11, len(frame) // 2, len(frame) - 5, len(frame) - 1):
        check(compressor, frame[:k])
    for k in (7, 8, 9, 10, 65551):
        f = bytearray(frame)
        f[k] ^= 0x40
        check(compressor, bytes(f))


def test_unlz4_index_many_blocks(compressor):
    """More blocks than the first index attempt takes (65536: the host retries with n / 5 + 2) and more
    candidates than the parallel index lists (it falls back to the one-lane walk)."""
    data = synth.enwik8_like(1 << 20, seed=76)
    frame = compressor.compress_blocks(data, 8, 65535)
    assert check(compressor, frame) == data
    frame = compressor.compress_blocks(data, 100, 65535)
    assert check(compressor, frame) == data


def test_unlz4_index_serial_and_parallel_agree(compressor, monkeypatch):
    """SZ4_UNLZ4_INDEX=0 keeps the one-lane walk (A/B): both index paths give the same output or both
    reject, on good, truncated and mutated frames."""
    import smallz4_amd
    monkeypatch.setenv("SZ4_UNLZ4_INDEX", "0")
    serial = smallz4_amd.Compressor(device=0)
    try:
        rng = np.random.default_rng(77)
        base = [compressor.compress_blocks(synth.enwik8_like(300000, seed=78), 4096, 65535),
                compressor.lz4(synth.enwik8_like(300000, seed=79), 9, b"", True)]
        for i in range(60):
            f = bytearray(base[i % 2])
            if i % 3 == 0:
                f = f[:int(rng.integers(0, len(f)))]
            else:
                k = int(rng.integers(4, len(f)))
                f[k] = int(rng.integers(0, 256))
            f = bytes(f)
            try:
                want = serial.unlz4(f)
            except NativeError:
                want = None
            if want is None:
                with pytest.raises(NativeError):
                    compressor.unlz4(f)
            else:
                assert compressor.unlz4(f) == want
    finally:
        serial.close()
