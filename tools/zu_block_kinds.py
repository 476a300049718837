#!/usr/bin/env python3
"""Diagnostic: stage times of 256 KiB blocks by zero-run layout (whole block of zeros, zeros to the end,
zeros from the start, a run inside), 64 blocks of each, each kind compressed on its own."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import smallz4_amd  # noqa: E402

bs = 262144
rng = np.random.default_rng(5)


def blocks(kind, nb=64):
    out = []
    for _ in range(nb):
        r = rng.integers(0, 256, bs, dtype=np.uint8)
        if kind == "whole":
            r[:] = 0
        elif kind == "to_end":
            r[100000:] = 0
        elif kind == "from_start":
            r[:160000] = 0
        elif kind == "inside":
            r[50000:200000] = 0
        out.append(r.tobytes())
    return b"".join(out)


comp = smallz4_amd.Compressor(device=0)
comp.set_timing(True)
for kind in sys.argv[1:] or ["whole", "to_end", "from_start", "inside"]:
    data = blocks(kind)
    t = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    cap = comp._lib.sz4_bound(len(data), bs)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    comp.compress_blocks_device(t.data_ptr(), len(data), out.data_ptr(), cap, bs, 65535)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    size = comp.compress_blocks_device(t.data_ptr(), len(data), out.data_ptr(), cap, bs, 65535)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"kind": kind, "ms": round(dt * 1e3, 2), "bytes": size,
                      "stages_ms": {k: round(v, 2) for k, v in comp.last_stage_ms().items()}}), flush=True)
