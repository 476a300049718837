#!/usr/bin/env python3
"""Debug: a tests/golden/blocks.json case on the GPU: which blocks differ from the reference, and for
the first one, the first positions where the finder's matches (after the match stage) differ from
the oracle's exhaustive search.  python tools/debug_blocks.py <case name>"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import inputs  # noqa: E402
import numpy as np  # noqa: E402
import smallz4_amd  # noqa: E402
from oracle import pyoracle  # noqa: E402

name = sys.argv[1]
case = [c for c in json.load(open(os.path.join(ROOT, "tests", "golden", "blocks.json")))["cases"] if c["name"] == name][0]
data = inputs.make(case["input"])
bs, chain = case["block_size"], case["max_chain"]
c = smallz4_amd.Compressor()
frame = c.compress_blocks(data, bs, chain)
pos, bad = 7, []
for i, (want, n) in enumerate(zip(case["block_sha256"], case["block_len"])):
    m = int.from_bytes(frame[pos:pos + 4], "little") & 0x7FFFFFFF
    if inputs.sha(frame[pos:pos + 4 + m]) != want:
        bad.append(i)
    pos += 4 + m
print("differing blocks", bad)
if bad:
    b = bad[0]
    blk = data[b * bs:(b + 1) * bs]
    c.debug_stop_after(3)
    c.compress_blocks(blk, bs, chain)
    gl, gd = c.debug_matches(len(blk))
    c.debug_stop_after(0)
    ol, od = pyoracle.oz_block_matches(blk, chain, 0)
    n = len(blk) - 11
    diff = np.flatnonzero((gl[:n] != ol[:n]) | ((gd[:n] != od[:n]) & (ol[:n] > 1)))
    print("block", b, "positions differing", len(diff))
    for p in diff[:12]:
        lo = max(0, p - 3)
        print(p, "gpu", int(gl[p]), int(gd[p]), "oracle", int(ol[p]), int(od[p]), "bytes", blk[lo:p + 8].hex())
