#!/usr/bin/env python3
"""Diagnostic: per-position matches of the finder stages (debug_stop_after(3)) against the oracle's
exhaustive search, on one synth input; prints the first differences with their context."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import smallz4_amd  # noqa: E402
from oracle import pyoracle  # noqa: E402
from smallz4_amd import synth  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "db"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 400000
bs = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
gen = {"db": synth._db_records, "xml": synth._xml_records, "exe": synth._opcodes}[kind]
data = gen(n, np.random.default_rng(77))
comp = smallz4_amd.Compressor()
comp.debug_stop_after(int(os.environ.get('STOP', '3')))
comp.compress_blocks(data, bs, 65535)
gl, gd = comp.debug_matches(len(data))
bad = 0
for o in range(0, len(data), bs):
    blk = data[o:o + bs]
    ol, od = pyoracle.oz_block_matches(blk, 65535, 0)
    m = len(blk) - 11
    if m <= 0:
        continue
    L, D = gl[o:o + m], gd[o:o + m]
    diff = np.nonzero((L != ol[:m]) | ((D != od[:m]) & (ol[:m] > 0)))[0]
    print(f"block {o // bs}: {len(diff)} positions differ", flush=True)
    for i in diff[:12]:
        print(f"  pos {i} (row off {(o + i) % 48}): gpu ({L[i]}, {D[i]}) oracle ({ol[i]}, {od[i]}); prev gpu ({L[i-1]},{D[i-1]}) oracle ({ol[i-1]},{od[i-1]})")
    bad += len(diff)
print("total differing positions:", bad)
