"""Parity of the HIP path (through the C ABI) with the oracle and the reference's golden
vectors.  Every comparison is byte-for-byte.  Run with -m gpu on an MI355X."""
import os
import time
import subprocess

import numpy as np
import pytest

import inputs
from oracle import pyoracle
from smallz4_amd import synth

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = bytes([0x04, 0x22, 0x4D, 0x18, 0x40, 0x70, 0xDF])


def expected_frame(data, bs, chain):
    # blocks are independent: the oracle runs them on threads (ctypes releases the GIL)
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=8) as ex:
        body = b"".join(ex.map(lambda o: pyoracle.oz_block(data[o:o + bs], chain), range(0, len(data), bs)))
    return HDR + body + b"\0\0\0\0"


# ---- independent blocks (the data-parallel path) --------------------------------------------
@pytest.mark.parametrize("chain", [0, 1, 2, 3, 4, 5, 6, 7, 8, 16, 65535])
def test_blocks_text_every_level(compressor, chain):
    data = synth.enwik8_like(1 << 20, seed=31)
    assert compressor.compress_blocks(data, 65536, chain) == expected_frame(data, 65536, chain)


@pytest.mark.parametrize("name,data", [
    ("random", synth.random_bytes(300000, seed=1)),
    ("alpha2", synth.small_alphabet(300000, k=2, seed=2)),
    ("alpha4", synth.small_alphabet(300000, k=4, seed=3)),
    ("runs", synth.runs(400000, seed=4, max_run=5000)),
    ("zeros", bytes(200000)),
    ("zeros_urandom", synth.zeros_urandom(600000, run=70000, seed=5)),
], ids=lambda v: v if isinstance(v, str) else "")
@pytest.mark.parametrize("chain", [7, 65535])
def test_blocks_shapes(compressor, name, data, chain):
    assert compressor.compress_blocks(data, 65536, chain) == expected_frame(data, 65536, chain)


@pytest.mark.parametrize("n", [1, 5, 11, 12, 13, 16, 100, 65535, 65536, 65537, 65548, 200001])
def test_blocks_edge_sizes(compressor, n):
    data = synth.enwik8_like(n, seed=n)
    for chain in (3, 65535):
        assert compressor.compress_blocks(data, 65536, chain) == expected_frame(data, 65536, chain)


@pytest.mark.parametrize("bs", [1000, 4096, 100000, 262144, 1 << 20, 4 << 20])
def test_blocks_other_block_sizes(compressor, bs):
    data = synth.enwik8_like(5 << 20, seed=7)
    assert compressor.compress_blocks(data, bs, 65535) == expected_frame(data, bs, 65535)


def test_blocks_empty(compressor):
    assert compressor.compress_blocks(b"", 65536, 65535) == HDR + b"\0\0\0\0"


def test_blocks_headers(compressor):
    data = synth.enwik8_like(200000, seed=8)
    bare = compressor.compress_blocks(data, 65536, 65535, header="none")
    full = compressor.compress_blocks(data, 65536, 65535)
    assert full == HDR + bare + b"\0\0\0\0"
    indep = compressor.compress_blocks(data, 65536, 65535, header="independent")
    import xxhash
    assert indep[:6] == bytes([4, 0x22, 0x4D, 0x18, 0x60, 0x40])
    assert indep[6] == (xxhash.xxh32(indep[4:6]).intdigest() >> 8) & 0xFF
    assert indep[7:] == full[7:]
    assert pyoracle.oz_unlz4(indep) == data


@pytest.mark.parametrize("name,data,bs,chains", [
    ("repeats64k", synth.repeats(400000, seed=21, unit=20000, mutate_every=3000), 65536, (7, 65535)),
    ("repeats256k", synth.repeats(600000, seed=22, unit=30000, mutate_every=9000), 262144, (7, 65535)),
    ("repeats1m", synth.repeats(700000, seed=25, unit=50000, mutate_every=30000), 1 << 20, (65535,)),
    ("runs256k", synth.runs(300000, seed=23, max_run=20000), 262144, (65535,)),
    ("zeros_urandom256k", synth.zeros_urandom(262144, seed=24), 262144, (65535,)),
], ids=lambda v: v if isinstance(v, str) else "")
def test_blocks_long_matches(compressor, name, data, bs, chains):
    """Matches of hundreds to tens of thousands of bytes: the parse's range minima (UP/DOWN), the
    repair pass across parse segments, the finder's early exit and pass-2 seed."""
    for chain in chains:
        assert compressor.compress_blocks(data, bs, chain) == expected_frame(data, bs, chain), chain


SILESIA_KINDS = {
    "db": synth._db_records, "xml": synth._xml_records, "exe": synth._opcodes,
    "image": synth._image16, "src": synth._source,
}


@pytest.mark.parametrize("kind", sorted(SILESIA_KINDS))
@pytest.mark.parametrize("bs", [65536, 262144])
def test_blocks_structured_content(compressor, kind, bs):
    """The Silesia-shaped generator's pieces on their own: fixed-width binary records (key groups of
    tens of thousands of candidates: k_find_big's left-maximal search and text-order prefix maximum,
    several segments per block at 256 KiB), XML records, an opcode stream, 16-bit images, source."""
    data = SILESIA_KINDS[kind](600000 if bs > 65536 else 400000, np.random.default_rng(77))
    for chain in (65535, 7) if kind != "db" else (65535,):
        assert compressor.compress_blocks(data, bs, chain) == expected_frame(data, bs, chain), chain


def test_zero_run_group_with_collision_ends(compressor):
    """A configs[4] block whose zero-run key group starts and ends with 16-bit hash collisions (random
    positions that hash like 0x00000000): k_find_big must still take it as a run-key group.  Round 3
    sent it to the class path (550 ms for one block, byte-identical but 700x slower); the oracle decides
    the bytes, the stage clock the path."""
    bs = 262144
    lo = 334495744  # 319 MiB into configs[4]'s rank-0 slice
    data = synth.zeros_urandom_range(lo, lo + bs, seed=10)
    compressor.set_timing(True)
    try:
        frame = compressor.compress_blocks(data, bs, 65535)
        find_long = compressor.last_stage_ms()["find_long"]
    finally:
        compressor.set_timing(False)
    assert frame[7:-4] == pyoracle.oz_block(data, 65535)
    assert find_long < 50.0, find_long


def test_blocks_silesia_mix_4m(compressor):
    """configs[2]'s shape: Silesia-shaped mixed content in 4 MiB independent blocks."""
    data = synth.silesia_like(5 << 20, seed=78)
    assert compressor.compress_blocks(data, 4 << 20, 65535) == expected_frame(data, 4 << 20, 65535)


def _blocks_golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "blocks.json")) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("case", _blocks_golden(), ids=lambda c: c["name"])
def test_blocks_golden_fixtures(compressor, case):
    """Full-size blocks the reference is too slow to redo inside a test (4 MiB blocks of binary
    records: ~2 minutes each at -9): every block's bytes against the reference's own output,
    recorded by tests/golden/make_blocks_golden.py.  Covers each Silesia kind at configs[2]'s 4 MiB,
    run-key groups (k_find_big's run bins) at 64 KiB / 256 KiB / 4 MiB, and configs[4]'s zeros/urandom
    layout at 256 KiB."""
    data = inputs.make(case["input"])
    assert inputs.sha(data) == case["input_sha256"]
    frame = compressor.compress_blocks(data, case["block_size"], case["max_chain"])
    assert len(frame) == case["frame_len"]
    pos, bad = 7, []
    for i, (want, n) in enumerate(zip(case["block_sha256"], case["block_len"])):
        if inputs.sha(frame[pos:pos + n]) != want:
            bad.append(i)
        pos += n
    assert not bad, f"blocks differing from the reference: {bad}"
    assert pyoracle.oz_unlz4(frame, cap=len(data) + 16) == data


def _skip_into_run(seed):
    """A long match that ends 10 bytes into a 100 KB zero run: at greedy/lazy levels the run's first
    positions are skipped, so the same-letter shortcut starts later than the run."""
    rng = np.random.default_rng(seed)
    r = rng.integers(1, 256, size=1000, dtype=np.uint8).tobytes()
    return synth.enwik8_like(3000, seed=seed) + r + bytes(10) + b"xyz" + r + bytes(100000) + synth.enwik8_like(20000, seed=seed + 1)


def _fixture(name):
    """A case of tests/golden/streams.json (the reference's own frame, made by make_streams_golden.py):
    (case, input).  For inputs with long zero runs, where the reference's chain walk is quadratic."""
    import json
    with open(os.path.join(ROOT, "tests", "golden", "streams.json")) as f:
        case = {c["name"]: c for c in json.load(f)["cases"]}[name]
    data = inputs.make(case["input"])
    assert inputs.sha(data) == case["input_sha256"]
    return case, data


def _matches_fixture(frame, case):
    return len(frame) == case["frame_len"] and inputs.sha(frame) == case["frame_sha256"]


@pytest.mark.parametrize("chain", [1, 2, 3, 4, 5, 6])
def test_greedy_lazy_long_runs(compressor, chain):
    """Greedy/lazy levels on same-letter runs > 65299 bytes: the parallel skip walk runs over the assumed
    shortcut intervals, k_lazy_check compares them with the ones its searches imply, and the pipeline reruns
    until they match the reference's loop (smallz4.h:631-643, 726-744).  Against the reference's own frames
    (tests/golden/streams.json)."""
    for name, data0, bs in ((f"gl_skip_into_run_l{chain}", _skip_into_run(40), 262144),
                            (f"gl_runs_a_l{chain}", synth.enwik8_like(30000, seed=41) + bytes(150000), 262144),
                            (f"gl_runs_b_l{chain}", bytes(70000) + synth.enwik8_like(5000, seed=42) + bytes(90000), 1 << 20)):
        case, data = _fixture(name)
        assert data == data0 and case["block_size"] == bs
        assert _matches_fixture(compressor.compress_blocks(data, bs, chain), case), name
    case, data = _fixture(f"gl_runs_4m_l{chain}")
    assert data == synth.enwik8_like((4 << 20) - 40000, seed=43) + bytes(140000) + synth.enwik8_like(10000, seed=44)
    assert _matches_fixture(compressor.lz4(data, chain), case)
    if chain in (1, 3, 5):
        # 21 MB through smallz4::lz4 with zero runs of 120 000 and 90 000 bytes (one across a 4 MiB block
        # boundary): every block with a run takes the parallel walk and its interval rounds (round 4 replayed
        # such blocks in one lane: 2.7-2.9 s; the reference on one CPU core: 0.9 s at -1, 2.2 s at -3; round 6:
        # 0.10 / 0.17 / 0.17 s at -1 / -3 / -5, tools/time_carry.py)
        case, data = _fixture(f"carry_state_l{chain}")
        compressor.lz4(data[:1 << 20], chain)
        t = time.perf_counter()
        out = compressor.lz4(data, chain)
        dt = time.perf_counter() - t
        print(f"carry_state_l{chain}: {len(data) / 1e6:.1f} MB in {dt:.3f} s")
        assert _matches_fixture(out, case)
        assert dt < 0.3, dt


def test_blocks_long_run_shortcut(compressor):
    # a same-letter run longer than MaxSameLetter inside one 256 KiB block (smallz4.h:631-643)
    for chain in (7, 8, 65535):
        case, data = _fixture(f"shortcut_256k_l{chain}")
        assert data == synth.enwik8_like(30000, seed=9) + bytes(150000) + synth.enwik8_like(82144, seed=10)
        assert _matches_fixture(compressor.compress_blocks(data, 262144, chain), case), chain


def test_finder_intermediate_matches(compressor):
    """k_find's per-position output equals the oracle's exhaustive search (stage 0)."""
    data = synth.enwik8_like(65536, seed=12)
    try:
        for chain in (1, 8, 65535):
            compressor.debug_stop_after(3)
            compressor.compress_blocks(data, 65536, chain)
            gl, gd = compressor.debug_matches(len(data))
            ol, od = pyoracle.oz_block_matches(data, chain, 0)
            n = len(data) - 11
            assert (gl[:n] == ol[:n]).all()
            assert (gd[:n][ol[:n] > 0] == od[:n][ol[:n] > 0]).all()
    finally:
        compressor.debug_stop_after(0)


def test_device_pointer_api_and_capacity(compressor):
    import torch
    data = synth.enwik8_like(300000, seed=13)
    t = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    cap = compressor._lib.sz4_bound(len(data), 65536)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    size = compressor.compress_blocks_device(t.data_ptr(), len(data), out.data_ptr(), cap, 65536, 65535)
    assert out[:size].cpu().numpy().tobytes() == expected_frame(data, 65536, 65535)
    from smallz4_amd._native import NativeError
    with pytest.raises(NativeError):
        compressor.compress_blocks_device(t.data_ptr(), len(data), out.data_ptr(), cap - 1, 65536, 65535)
    sizes = compressor.last_block_sizes(5)
    assert sum(sizes) == size - 11


def test_large_roundtrip_property(compressor):
    """100 MB: the frame decodes back to the input, every block's size word matches its body."""
    data = synth.enwik8_like(100_000_000, seed=14)
    frame = compressor.compress_blocks(data, 65536, 65535)
    assert pyoracle.oz_unlz4(frame, cap=len(data) + 16) == data
    pos, blocks = 7, 0
    while pos < len(frame) - 4:
        word = int.from_bytes(frame[pos:pos + 4], "little")
        pos += 4 + (word & 0x7FFFFFFF)
        blocks += 1
    assert pos == len(frame) - 4 and blocks == (len(data) + 65535) // 65536


# ---- whole-stream smallz4::lz4 semantics -----------------------------------------------------
def test_golden_vectors_on_gpu(compressor, golden):
    for case in golden:
        data = inputs.make(case["input"])
        dictionary = inputs.make(case["dict"]) if "dict" in case else b""
        frame = compressor.lz4(data, case["level"], dictionary, bool(case["legacy"]))
        assert inputs.sha(frame) == case["out_sha256"], (case["name"], case["level"], case["legacy"])


@pytest.mark.parametrize("legacy", [False, True])
@pytest.mark.parametrize("chain", [2, 6, 65535])
def test_stream_multiblock(compressor, chain, legacy):
    data = synth.enwik8_like(9 << 20, seed=15)
    assert compressor.lz4(data, chain, b"", legacy) == pyoracle.oz_lz4(data, chain, b"", legacy)


def test_stream_run_across_block_boundary(compressor):
    M = 4 << 20
    data = synth.enwik8_like(M - 30000, seed=16) + bytes(100000) + synth.enwik8_like(200000, seed=17)
    assert compressor.lz4(data, 65535) == pyoracle.oz_lz4(data, 65535)


@pytest.mark.parametrize("chain", [3, 6, 9, 65535])
def test_dictionary_mode(compressor, chain):
    """Dictionary mode reproduces the reference byte for byte, including its misaligned chain slots
    (DESIGN.md section 3.7): the data-parallel snapshot reads of sz4_dict.hip for modern frames, the
    in-order replay (k_dict_matches) for legacy ones; the parse and assembly are shared."""
    cases = [
        (synth.enwik8_like(60000, seed=50), synth.enwik8_like(20000, seed=51), False),
        (synth.enwik8_like(40000, seed=52), synth.enwik8_like(70000, seed=53), False),
        (bytes(20) + synth.enwik8_like(30000, seed=54), b"short dictionary", False),
        (synth.enwik8_like(30000, seed=55), synth.enwik8_like(5000, seed=56), True),
        # runs and periodic data: long phase-2 extensions, hash-collision walks, duplicate re-insertions
        (bytes(20000) + synth.enwik8_like(20000, seed=57) * 3, b"\0" * 500 + b"xyz" * 3000, False),
        (b"abcd" * 5000 + synth.random_bytes(50000, seed=58), synth.random_bytes(70000, seed=59), False),
        (b"", synth.enwik8_like(1000, seed=60), False),
        (b"tiny", synth.enwik8_like(1000, seed=61), False),
    ]
    for data, dictionary, legacy in cases:
        assert compressor.lz4(data, chain, dictionary, legacy) == pyoracle.oz_lz4(data, chain, dictionary, legacy)


def test_cpp_dropin_program(tmp_path):
    exe = tmp_path / "dropin_demo"
    subprocess.run(["hipcc", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "dropin_demo.cpp"), "-L", os.path.join(ROOT, "smallz4_amd", "lib"),
                    "-lsmallz4_amd", "-Wl,-rpath," + os.path.join(ROOT, "smallz4_amd", "lib"), "-o", str(exe)],
                   check=True)
    data = synth.enwik8_like(5 << 20, seed=18)
    for level, legacy in ((9, 0), (6, 1)):
        r = subprocess.run([str(exe), str(level), str(legacy)], input=data, capture_output=True, check=True)
        chain = 65535 if level == 9 else level
        assert r.stdout == pyoracle.oz_lz4(data, chain, b"", bool(legacy))


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "smallz4_on_amd")),
                    reason="reference CLI not rebuilt against the drop-in header")
def test_reference_cli_rebuilt_on_dropin(tmp_path):
    """The reference's own smallz4.cpp, compiled unchanged against include/compat/smallz4.h,
    produces the same files as the reference binary (both built by oracle/Makefile)."""
    amd = os.path.join(ROOT, "oracle", "_ref", "smallz4_on_amd")
    ref = os.path.join(ROOT, "oracle", "_ref", "smallz4")
    src = tmp_path / "in.txt"
    src.write_bytes(synth.enwik8_like(6 << 20, seed=19))
    dic = tmp_path / "dict.txt"
    dic.write_bytes(synth.enwik8_like(30000, seed=20))
    for flags in (["-9"], ["-6"], ["-2"], ["-0"], ["-9", "-l"], ["-D", str(dic), "-9"]):
        a, b = tmp_path / "a.lz4", tmp_path / "b.lz4"
        subprocess.run([amd, "-f", *flags, str(src), str(a)], check=True)
        subprocess.run([ref, "-f", *flags, str(src), str(b)], check=True)
        assert a.read_bytes() == b.read_bytes(), flags
