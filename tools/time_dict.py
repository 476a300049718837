#!/usr/bin/env python3
"""Dictionary-mode throughput (the data-parallel finder of sz4_dict.hip) through
sz4_lz4 (host buffers), next to the same input without a dictionary; run under rocprofv3 --kernel-trace
--stats for the per-kernel split.

    python tools/time_dict.py [MB]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import smallz4_amd  # noqa: E402
from smallz4_amd import synth  # noqa: E402

mb = float(sys.argv[1]) if len(sys.argv) > 1 else 8
data = synth.enwik8_like(int(mb * 1e6), seed=30)
dictionary = synth.enwik8_like(65536, seed=31)
comp = smallz4_amd.Compressor()
for chain in (65535, 6):  # first calls grow the context's buffers to this input
    for dic in (b"", dictionary):
        comp.lz4(data, chain, dic)
for chain in (65535, 6):
    for dic in (b"", dictionary):
        t = time.perf_counter()
        out = comp.lz4(data, chain, dic)
        dt = time.perf_counter() - t
        print(json.dumps({"chain": chain, "dictionary_bytes": len(dic), "input_bytes": len(data),
                          "MB/s": round(len(data) / dt / 1e6, 2), "ratio": round(len(out) / len(data), 4)}), flush=True)
