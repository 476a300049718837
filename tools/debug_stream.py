#!/usr/bin/env python3
"""Debug: the golden vectors through the stream path (sz4_lz4) with one 4 MiB block per chunk, in one
warm context; for a failing case, the first differing byte, and the same case in a fresh context."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import inputs  # noqa: E402
import smallz4_amd  # noqa: E402
from oracle import pyoracle  # noqa: E402

M = 4 << 20
cases = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))["cases"]
c = smallz4_amd.Compressor()
c.set_stream_chunk(M)
for case in cases:
    data = inputs.make(case["input"])
    dic = inputs.make(case["dict"]) if "dict" in case else b""
    got = c.lz4(data, case["level"], dic, bool(case["legacy"]))
    if inputs.sha(got) == case["out_sha256"]:
        continue
    want = pyoracle.oz_lz4(data, case["level"], dic, bool(case["legacy"]))
    d = next((i for i in range(min(len(got), len(want))) if got[i] != want[i]), None)
    f = smallz4_amd.Compressor()
    f.set_stream_chunk(M)
    fresh = f.lz4(data, case["level"], dic, bool(case["legacy"]))
    print("FAIL", case["name"], case["level"], case["legacy"], "len", len(got), len(want), "first diff", d,
          "fresh ok", fresh == want, flush=True)
print("done")
