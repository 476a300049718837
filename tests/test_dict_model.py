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
