#!/usr/bin/env python3
"""Diagnostic: configs[4]'s generator, one 256 KiB block per call from <start MiB>, <count> blocks;
prints the blocks whose find_long stage exceeds 2 ms (and saves the slowest one to /tmp/zu_slow.bin)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import smallz4_amd  # noqa: E402
from smallz4_amd import synth  # noqa: E402

bs = 262144
start = int(float(sys.argv[1]) * (1 << 20))
count = int(sys.argv[2])
comp = smallz4_amd.Compressor(device=0)
comp.set_timing(True)
worst = (0.0, None)
for b in range(count):
    lo = start + b * bs
    data = synth.zeros_urandom_range(lo, lo + bs, seed=10)
    comp.compress_blocks(data, bs, 65535)
    fl = comp.last_stage_ms()["find_long"]
    if fl > 2.0:
        print(json.dumps({"block_at": lo, "find_long_ms": round(fl, 2)}), flush=True)
    if fl > worst[0]:
        worst = (fl, data)
if worst[1] is not None:
    open(os.path.join(ROOT, "gpurun_out", "zu_slow.bin"), "wb").write(worst[1])
print(json.dumps({"worst_find_long_ms": round(worst[0], 2)}), flush=True)
