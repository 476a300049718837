#!/usr/bin/env python3
"""Diagnostic: configs[4]'s rank-0 slice (zeros/urandom, 256 KiB blocks) compressed piece by piece, to
find the regions whose find_long stage is slow.  python tools/zu_pieces.py [piece MiB] [end MiB] [start MiB]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import smallz4_amd  # noqa: E402
from smallz4_amd import synth  # noqa: E402

piece = int(float(sys.argv[1]) * (1 << 20)) if len(sys.argv) > 1 else 256 << 20
total = int(float(sys.argv[2]) * (1 << 20)) if len(sys.argv) > 2 else 1280 << 20
start = int(float(sys.argv[3]) * (1 << 20)) if len(sys.argv) > 3 else 0
bs = 262144
comp = smallz4_amd.Compressor(device=0)
comp.set_timing(True)
for lo in range(start, total, piece):
    hi = min(lo + piece, total)
    data = synth.zeros_urandom_range(lo, hi, seed=10)
    x = np.frombuffer(data, dtype=np.uint8)
    t = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    cap = comp._lib.sz4_bound(len(data), bs)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    comp.compress_blocks_device(t.data_ptr(), len(data), out.data_ptr(), cap, bs, 65535)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    comp.compress_blocks_device(t.data_ptr(), len(data), out.data_ptr(), cap, bs, 65535)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # longest zero run in the piece
    z = np.concatenate(([0], (x == 0).astype(np.int8), [0]))
    d = np.diff(z)
    runs = np.flatnonzero(d == -1) - np.flatnonzero(d == 1)
    print(json.dumps({"lo_MiB": lo / (1 << 20), "hi_MiB": hi / (1 << 20), "ms": round(dt * 1e3, 2),
                      "stages_ms": {k: round(v, 2) for k, v in comp.last_stage_ms().items()},
                      "zero_runs": int(len(runs)), "max_zero_run": int(runs.max()) if len(runs) else 0,
                      "runs_over_256k": int((runs > bs).sum())}), flush=True)
