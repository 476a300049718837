"""The oracle (C restatement of the reference, oracle/smallz4_oracle.c) is pinned here:
against the golden vectors produced by the reference itself (tests/golden/golden.json,
tests/golden/make_golden.py) and, when the reference tree was present at build time,
against the reference compiled in place (oracle/_ref/)."""
import os
import subprocess

import numpy as np
import pytest

import inputs
from oracle import pyoracle
from smallz4_amd import synth

SLOW = {"zu256k", "text9m", "text9m_cut", "tail5", "tail13", "zeros_across_blocks", "alpha2", "alpha4",
        "runs100k", "zeros64k", "zeros70k"}


def _cases(golden, slow):
    return [c for c in golden if (c["name"] in SLOW) == slow]


def _check(case):
    data = inputs.make(case["input"])
    assert inputs.sha(data) == case["input_sha256"], "fixture generator changed"
    dic = inputs.make(case["dict"]) if "dict" in case else b""
    frame = pyoracle.oz_lz4(data, case["level"], dic, bool(case["legacy"]))
    assert len(frame) == case["out_len"]
    assert inputs.sha(frame) == case["out_sha256"]
    if "out_hex" in case:
        assert frame.hex() == case["out_hex"]


def test_golden_fast(golden):
    cases = _cases(golden, slow=False)
    assert len(cases) > 40
    for case in cases:
        _check(case)


@pytest.mark.slow
def test_golden_slow(golden):
    for case in _cases(golden, slow=True):
        _check(case)


def test_golden_covers_every_level_and_mode(golden):
    levels = {c["level"] for c in golden}
    assert set(range(0, 9)) | {65535} <= levels
    assert any(c["legacy"] for c in golden)
    assert any("dict" in c for c in golden)
    assert any(c["input_len"] > (4 << 20) for c in golden)   # multi-block streams
    assert any(c["input_len"] == 0 for c in golden)


def test_blocks_golden_inputs_unchanged():
    """tests/golden/blocks.json (independent-block fixtures of the reference, checked on the GPU by
    test_gpu.py::test_blocks_golden_fixtures): the generators still produce the recorded inputs."""
    import json
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "blocks.json")) as f:
        cases = json.load(f)["cases"]
    assert {"db_4m", "xml_4m", "exe_4m", "image_4m", "src_4m", "text_4m", "zu_256k"} <= {c["name"] for c in cases}
    for case in cases:
        data = inputs.make(case["input"])
        assert inputs.sha(data) == case["input_sha256"], case["name"]
        nb = (len(data) + case["block_size"] - 1) // case["block_size"]
        assert len(case["block_sha256"]) == len(case["block_len"]) == nb
        assert case["frame_len"] == 11 + sum(case["block_len"])


@pytest.mark.skipif(not pyoracle.ref_available(), reason="reference not compiled (oracle/_ref)")
@pytest.mark.parametrize("seed", range(6))
def test_oracle_matches_reference_random(seed):
    rng = np.random.default_rng(100 + seed)
    for _ in range(6):
        n = int(rng.integers(0, 40000))
        kind = int(rng.integers(0, 4))
        if kind == 0:
            data = synth.enwik8_like(n, seed=int(rng.integers(1 << 30)))
        elif kind == 1:
            data = synth.small_alphabet(n, k=int(rng.integers(1, 5)), seed=seed)
        elif kind == 2:
            data = synth.runs(n, seed=seed, max_run=200)
        else:
            data = synth.random_bytes(n, seed=seed)
        level = int(rng.choice([0, 1, 2, 3, 4, 5, 6, 7, 8, 13, 200, 65535]))
        legacy = bool(rng.integers(0, 2)) and level != 0
        dic = synth.enwik8_like(int(rng.integers(1, 70000)), seed=seed) if rng.integers(0, 4) == 0 else b""
        assert pyoracle.oz_lz4(data, level, dic, legacy) == pyoracle.ref_lz4(data, level, dic, legacy)


@pytest.mark.parametrize("level", [1, 4, 7, 65535])
def test_roundtrip_decoder(level):
    for data in [b"", b"x", synth.enwik8_like(150000, seed=4), synth.runs(80000, seed=1, max_run=500),
                 synth.random_bytes(20000)]:
        for legacy in (False, True):
            assert pyoracle.oz_unlz4(pyoracle.oz_lz4(data, level, b"", legacy)) == data


@pytest.mark.skipif(not os.path.exists(pyoracle.REF_CAT), reason="reference decoder not compiled")
def test_reference_decoder_accepts_oracle_frames(tmp_path):
    data = synth.enwik8_like(300000, seed=5)
    f = tmp_path / "x.lz4"
    f.write_bytes(pyoracle.oz_lz4(data, 65535))
    out = subprocess.run([pyoracle.REF_CAT, str(f)], capture_output=True, check=True).stdout
    assert out == data


def test_reference_dictionary_mode_is_not_decodable(golden):
    """Pins a reference defect the port reproduces: with a dictionary, chain entries are written
    at block-relative slots but read at absolute ones (smallz4.h:656 vs 190/694), so the frame
    can reference wrong bytes.  The golden vector itself comes from the reference."""
    case = next(c for c in golden if c["name"] == "dict30k" and c["level"] == 65535)
    data, dic = inputs.make(case["input"]), inputs.make(case["dict"])
    frame = pyoracle.oz_lz4(data, 65535, dic)
    assert inputs.sha(frame) == case["out_sha256"]
    assert pyoracle.oz_unlz4(frame, dic) != data


def test_block_matches_stages():
    data = synth.enwik8_like(65536, seed=2)
    l0, d0 = pyoracle.oz_block_matches(data, 65535, 0)
    l2, d2 = pyoracle.oz_block_matches(data, 65535, 2)
    assert ((l0 == 0) | (l0 >= 4)).all()
    assert (d0[l0 >= 4] > 0).all()
    assert (l2[: len(data) - 5] >= 1).all()
    # chosen lengths never exceed the longest available match
    assert (l2[l2 > 1] <= l0[l2 > 1]).all()


def test_oz_block_is_frame_body():
    data = synth.enwik8_like(65536, seed=3)
    frame = pyoracle.oz_lz4(data, 65535)
    assert pyoracle.oz_block(data, 65535) == frame[7:-4]


def _flag_frame(flags, frame):
    """Re-wrap the blocks of a 7-byte-header modern frame with descriptor FLG `flags` (content size,
    dictionary ID, block and content checksums filled with arbitrary bytes: the decoder skips them)."""
    import struct
    pos, body = 7, b""
    while True:
        word = int.from_bytes(frame[pos:pos + 4], "little")
        pos += 4
        if word == 0:
            break
        n = word & 0x7FFFFFFF
        body += frame[pos - 4:pos + n] + (b"\xDE\xAD\xBE\xEF" if flags & 16 else b"")
        pos += n
    hdr = frame[:4] + bytes([flags, 0x70]) + (struct.pack("<Q", 7) if flags & 8 else b"") + \
        (b"\x11\x22\x33\x44" if flags & 1 else b"") + b"\xAB"
    return hdr + body + b"\0\0\0\0" + (b"\x01\x02\x03\x04" if flags & 4 else b"")


@pytest.mark.skipif(not os.path.exists(pyoracle.REF_CAT), reason="reference decoder not compiled")
def test_decoder_oracle_matches_reference_binary(tmp_path):
    """oz_unlz4 -- the checker of the device decoder -- against the reference's own smallz4cat: the
    same bytes on valid frames (descriptor fields, stored and legacy blocks, a >= 64 KiB dictionary),
    and both reject signature, version, truncation and offset-0 errors.  Not compared: references
    before the history (the reference reads uninitialised memory) and tokens that run past their
    block (the reference reads on into the next block; oz_unlz4 and the device reject them)."""
    data = synth.enwik8_like(150000, seed=80) + synth.random_bytes(30000, seed=81)
    dic = synth.enwik8_like(70000, seed=82)
    (tmp_path / "d").write_bytes(dic)
    m = pyoracle.oz_lz4(data, 9)
    valid = [(m, None), (pyoracle.oz_lz4(data, 0), None), (pyoracle.oz_lz4(data, 6, b"", True), None),
             (_flag_frame(0x5D, m), None), (_flag_frame(0x48, m), None),
             (pyoracle.oz_lz4(data[:60000], 7, dic), str(tmp_path / "d"))]
    for frame, d in valid:
        ref = subprocess.run([pyoracle.REF_CAT] + (["-D", d] if d else []), input=frame, capture_output=True)
        assert ref.returncode == 0
        assert ref.stdout == pyoracle.oz_unlz4(frame, dic if d else b"")
    hdr = bytes([4, 0x22, 0x4D, 0x18, 0x40, 0x70, 0xDF])
    bad = [b"\x00\x22\x4d\x18" + m[4:], bytes([4, 0x22, 0x4D, 0x18, 0x00, 0x70, 0xDF, 0, 0, 0, 0]),
           hdr + b"\x04\0\0\0" + b"\x10a\x00\x00" + b"\0\0\0\0", m[:len(m) // 2], m[:-4], m[:5]]
    for frame in bad:
        ref = subprocess.run([pyoracle.REF_CAT], input=frame, capture_output=True)
        assert ref.returncode == 1
        with pytest.raises(ValueError):
            pyoracle.oz_unlz4(frame)


@pytest.mark.skipif(not os.path.exists(pyoracle.REF_CAT), reason="reference decoder not compiled")
def test_reference_legacy_level0_loses_data():
    """Pins a reference defect: a legacy frame at level 0 carries an empty block (no literals), and
    the reference's smallz4cat decodes it to nothing; oz_unlz4 and the device decoder agree."""
    frame = pyoracle.ref_lz4(b"abcdefgh" * 100, 0, b"", True)
    assert frame == bytes.fromhex("02214c1800000000")
    out = subprocess.run([pyoracle.REF_CAT], input=frame, capture_output=True, check=True).stdout
    assert out == b"" == pyoracle.oz_unlz4(frame)


def test_oracle_matches_stream_fixtures():
    """tests/golden/streams.json (whole-stream fixtures of the reference, checked on the GPU by
    test_stream.py): the C restatement reproduces the cases the reference itself finishes in about a
    second (dictionary runs at -6 / -3, legacy frames with a dictionary at -3)."""
    import json
    import inputs
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "streams.json")) as f:
        # (the dictionary cases: the oracle restates greedy/lazy runs far slower than the reference runs them)
        cases = [c for c in json.load(f)["cases"] if c["ref_seconds"] <= 1.5 and c["name"].startswith("dict_")]
    assert len(cases) >= 3
    for c in cases:
        data = inputs.make(c["input"])
        assert inputs.sha(data) == c["input_sha256"], c["name"]
        if c.get("kind") == "blocks":
            bs = c["block_size"]
            out = bytes([0x04, 0x22, 0x4D, 0x18, 0x40, 0x70, 0xDF]) + b"".join(
                pyoracle.oz_block(data[o:o + bs], c["max_chain"]) for o in range(0, len(data), bs)) + bytes(4)
        else:
            dic = inputs.make(c["dictionary"]) if c["dictionary"] else b""
            out = pyoracle.oz_lz4(data, c["max_chain"], dic, c["legacy"])
        assert len(out) == c["frame_len"] and inputs.sha(out) == c["frame_sha256"], c["name"]
