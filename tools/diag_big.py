#!/usr/bin/env python3
"""Diagnostic: k_find_big's counters from a SZ4_DIAG=4 build of the library (tools/build_diag.sh 4):
LM chunks (waves), candidate steps of the bin scans and of the fallback scans, lanes by kind."""
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

kind = sys.argv[1] if len(sys.argv) > 1 else "db"
mb = float(sys.argv[2]) if len(sys.argv) > 2 else 16
bs = int(sys.argv[3]) if len(sys.argv) > 3 else 4 << 20
n = int(mb * 1e6)
data = synth._silesia_piece((kind, n, 2, 7)) if kind != "silesia" else synth.silesia_like(n, seed=2, workers=8)
comp = smallz4_amd.Compressor()
lib = comp._lib
lib.sz4_diag_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
lib.sz4_diag_clear.argtypes = []
lib.sz4_diag_clear()
comp.compress_blocks(data, bs, 65535)
buf = np.zeros(16, dtype=np.uint64)
assert lib.sz4_diag_read(buf.ctypes.data, buf.size) == 0
names = ["waves", "scan_steps", "fb_waves", "fb_steps", "fb_lanes", "start_lanes", "interior_lanes", "nonrun_lanes",
         "interior_at_limit", "ext_iters"]
print(kind, mb, "MB", {k: int(v) for k, v in zip(names, buf)})
