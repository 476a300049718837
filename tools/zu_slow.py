#!/usr/bin/env python3
"""Diagnostic: compress one 256 KiB block of configs[4]'s generator (at 319 MiB: its zero-run group
starts and ends with hash collisions) a few times with stage times;
with SMALLZ4_AMD_LIB pointing at a SZ4_DIAG=6 build also k_find_big's counters."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import smallz4_amd  # noqa: E402
from oracle import pyoracle  # noqa: E402  (checker)

from smallz4_amd import synth  # noqa: E402

data = synth.zeros_urandom_range(334495744, 334495744 + 262144, seed=10)
comp = smallz4_amd.Compressor()
comp.set_timing(True)
diag = "diag" in os.environ.get("SMALLZ4_AMD_LIB", "")
lib = comp._lib
if diag:
    lib.sz4_diag_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
for r in range(3):
    if diag:
        lib.sz4_diag_clear()
    out = comp.compress_blocks(data, 262144, 65535)
    rec = {"rep": r, "stages_ms": {k: round(v, 2) for k, v in comp.last_stage_ms().items()}}
    if diag:
        buf = np.zeros(28, dtype=np.uint64)
        lib.sz4_diag_read(buf.ctypes.data, 28)
        rec["diag"] = [int(v) for v in buf]
    print(json.dumps(rec), flush=True)
exp = bytes([0x04, 0x22, 0x4D, 0x18, 0x40, 0x70, 0xDF]) + pyoracle.oz_block(data, 65535) + b"\0\0\0\0"
print(json.dumps({"equal_oracle": out == exp}), flush=True)
