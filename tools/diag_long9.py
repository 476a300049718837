#!/usr/bin/env python3
"""Diagnostic: k_find_long9's counters from a SZ4_DIAG=5 build (tools/build_diag.sh 5): best_of calls,
its 64-candidate steps, best_lane calls, their candidate steps, repair re-walks; on zeros/urandom."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SMALLZ4_AMD_LIB"] = os.path.join(ROOT, "smallz4_amd", "lib", "libsmallz4_amd_diag.so")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import smallz4_amd  # noqa: E402
from smallz4_amd import synth  # noqa: E402

mb = float(sys.argv[1]) if len(sys.argv) > 1 else 32
n = int(mb * 1e6) // 262144 * 262144
data = synth.zeros_urandom_range(0, n, seed=10)
comp = smallz4_amd.Compressor()
lib = comp._lib
lib.sz4_diag_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
lib.sz4_diag_clear()
comp.set_timing(True)
comp.compress_blocks(data, 262144, 65535)
buf = np.zeros(64 + 3 * 512, dtype=np.uint64)
lib.sz4_diag_read(buf.ctypes.data, len(buf))
print(mb, "MB", dict(zip(["best_of", "of_steps", "best_lane", "lane_steps", "rewalks", "marked", "interval", "cmp_words"], [int(x) for x in buf[:8]])),
      comp.last_stage_ms())
if len(sys.argv) > 2:
    for k in range(min(512, int(buf[15]))):
        rel, w, md = int(buf[64 + 3 * k]), int(buf[65 + 3 * k]), int(buf[66 + 3 * k])
        print(rel, f"{w:016x}", md & 0xFFFF, md >> 32)
