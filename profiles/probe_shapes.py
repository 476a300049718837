#!/usr/bin/env python3
"""Per-stage device times of the compressor on the pieces of the Silesia-shaped generator (and any
other synth generator), one kind at a time: which content makes which kernel slow.

    python profiles/probe_shapes.py [--mb 8] [--block-size 4194304] [--kinds text,xml,exe,db,image,src]

Prints one JSON line per kind: MB/s of the whole call, the stage times (HIP events), the ratio.
Diagnostic only (no parity check; the parity tests cover these generators)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from smallz4_amd import synth  # noqa: E402

KINDS = {
    "text": lambda n, rng: synth.enwik8_like(n, seed=int(rng.integers(0, 1 << 30))),
    "xml": lambda n, rng: synth._xml_records(n, rng),
    "exe": lambda n, rng: synth._opcodes(n, rng),
    "db": lambda n, rng: synth._db_records(n, rng),
    "image": lambda n, rng: synth._image16(n, rng),
    "src": lambda n, rng: synth._source(n, rng),
    "silesia": lambda n, rng: synth.silesia_like(n, seed=2),
    "zu": lambda n, rng: synth.zeros_urandom_range(0, n, seed=10),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, default=8.0)
    ap.add_argument("--block-size", type=int, default=4 << 20)
    ap.add_argument("--level", type=int, default=9)
    ap.add_argument("--kinds", default="text,xml,exe,db,image,src")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import torch
    import smallz4_amd
    comp = smallz4_amd.Compressor(device=0)
    comp.set_timing(True)
    chain = smallz4_amd.level_to_chain(a.level)
    n = int(a.mb * 1e6)
    for kind in a.kinds.split(","):
        data = KINDS[kind](n, np.random.default_rng(7))
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
        cap = comp._lib.sz4_bound(n, a.block_size)
        out = torch.empty(cap, dtype=torch.uint8, device="cuda")
        best, stages, size = None, None, 0
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            size = comp.compress_blocks_device(t.data_ptr(), n, out.data_ptr(), cap, a.block_size, chain)
            dt = time.perf_counter() - t0
            if best is None or dt < best:
                best, stages = dt, comp.last_stage_ms()
        print(json.dumps({"kind": kind, "bytes": n, "block_size": a.block_size, "level": a.level,
                          "MB/s": round(n / best / 1e6, 1), "ratio": round(size / n, 4),
                          "stages_ms": {k: round(v, 3) for k, v in stages.items()}}), flush=True)


if __name__ == "__main__":
    main()
