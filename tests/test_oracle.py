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
