#!/usr/bin/env python3
"""Diagnostic: k_find_big's phase clocks and counters from a SZ4_DIAG=6 build (tools/build_diag.sh 6)."""
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

kind = sys.argv[1]
mb = float(sys.argv[2])
bs = int(sys.argv[3])
n = int(mb * 1e6) // bs * bs
data = synth.zeros_urandom_range(0, n, seed=10) if kind == "zu" else synth._silesia_piece((kind, n, 2, 7))
comp = smallz4_amd.Compressor()
lib = comp._lib
lib.sz4_diag_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
comp.compress_blocks(data[:bs * 4], bs, 65535)
lib.sz4_diag_clear()
comp.set_timing(True)
comp.compress_blocks(data, bs, 65535)
buf = np.zeros(28, dtype=np.uint64)
lib.sz4_diag_read(buf.ctypes.data, 28)
names = ["detect", "window", "A", "A2scan", "phase3_wait", "C_run", "loop_top", "class_path", "run_targets",
         "bucket_it", "walk_it", "coop_steps", "pieces", "class_groups", "run_groups", "segments", "bad_threads", "mixed", "too_many_runs",
         "coll_targets", "coll_steps", "w_local", "w_coop", "w_coll", "ng0", "ng_over", "B_unresolved", "U_left"]
print(kind, mb, bs, {k: int(v) for k, v in zip(names, buf)}, {k: round(v, 2) for k, v in comp.last_stage_ms().items()})
