"""CPU model checks of the data-parallel dictionary mode (smallz4_amd/csrc/sz4_dict.hip, DESIGN.md
section 3.7), restated in Python by tools/dict_model.py:
  * the snapshot-read algorithm (previousHash by a (hash, position) sort, chain slots read from the
    latest insertion per slot, previousExact and findLongestMatch per position) gives the same match
    arrays and final chain tables as the in-order replay of the reference's loop (smallz4.h:603-760),
    at a block size small enough for Python (a multiple of 65536 keeps the dictionary's alignment);
  * the speculative per-sub-segment greedy/lazy walk with its repair (k_dict_lz_*) searches exactly the
    positions the reference's skip bookkeeping searches (smallz4.h:726-744), length-1 searches included.
The GPU kernels themselves are checked against the oracle in test_gpu.py / test_stream.py."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import dict_model  # noqa: E402


def test_lazy_walk_model_matches_serial_bookkeeping():
    rng = random.Random(3)
    for _ in range(500):
        n = rng.randint(1, 400)
        p = rng.random()
        linked = [rng.random() < p for _ in range(n)]
        lengths = [rng.choice([1, 1, 2, 3, 4, 9, 50, 300]) for _ in range(n)]
        assert dict_model.lz_serial(linked, lengths) == dict_model.lz_spec(linked, lengths)


def test_snapshot_model_matches_in_order_replay():
    data, blocks, dict_back = dict_model.make_case(131072, 140000, 20000, 4)
    assert len(blocks) == 2  # a block boundary inside the input: reads cross it
    a = dict_model.serial(data, blocks, dict_back, 65535)
    b = dict_model.parallel(data, blocks, dict_back, 65535)
    assert a[0] == b[0] and a[1] == b[1]  # match lengths and distances
    assert a[2] == b[2] and a[3] == b[3]  # the chain tables carried to a next chunk


def test_shortcut_rounds_model_matches_in_order_replay(monkeypatch):
    """The same-letter shortcut in dictionary mode (smallz4.h:631-643): rounds of the data-parallel
    algorithm under assumed shortcut positions, each replaced by the positions its results imply, end
    on the reference's match arrays and chain tables (k_dict_sc_bits / k_dict_sc and the host loop).
    MaxSameLetter is lowered to 200 so that Python can walk the runs (the round logic, not the
    constant, is under test); runs before, inside and across a block boundary."""
    from smallz4_amd import synth
    monkeypatch.setattr(dict_model, "SAME", 200)
    t = lambda n, s: synth.enwik8_like(n, seed=s)  # noqa: E731
    body = t(10000, 3) + b"a" * 1200 + t(3000, 4) + b"a" * 250 + t(2000, 5) + bytes(2000) + t(115000, 6) + \
        b"x" * 3000 + t(20000, 7)
    dic = t(5000, 8)
    W = dict_model.W
    data = (b"\0" * W + dic)[-W:] + body + b"\0" * 16
    blocks, s = [], W
    while s < W + len(body):
        blocks.append((s, min(s + 131072, W + len(body))))
        s += 131072
    assert len(blocks) == 2
    a = dict_model.serial(data, blocks, len(dic), 65535)
    rounds = []
    b = dict_model.parallel_sc(data, blocks, len(dic), 65535, rounds)
    assert sum(1 for p in a[0] if a[1].get(p) == 1 and a[0][p] > 200) > 1000  # the shortcut fired
    assert a == b and rounds[0] >= 2
