#!/usr/bin/env python3
"""Times the device decoder (sz4_unlz4_device) on one bench shape's frame -- run under
`rocprofv3 --kernel-trace --stats` for the per-kernel picture.
    python3 tools/prof_unlz4.py silesia|text4m|enwik8|zu [--mb MB] [--reps N]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

import smallz4_amd  # noqa: E402
from prof_shape import SHAPES, shape_data  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("shape", choices=sorted(SHAPES))
    ap.add_argument("--mb", type=float, default=None)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    full, bs, _ = SHAPES[a.shape]
    n = int(a.mb * 1e6) if a.mb else full
    arr = shape_data(a.shape, n).copy()
    dev = torch.device("cuda:0")
    t_in = torch.from_numpy(arr).to(dev)
    comp = smallz4_amd.Compressor()
    cap = comp._lib.sz4_bound(n, bs)
    fr = torch.empty(cap, dtype=torch.uint8, device=dev)
    size = comp.compress_blocks_device(t_in.data_ptr(), n, fr.data_ptr(), cap, bs, 65535)
    out = torch.empty(n, dtype=torch.uint8, device=dev)
    got = comp.unlz4_device(fr.data_ptr(), size, out.data_ptr(), n)
    torch.cuda.synchronize()
    assert got == n and torch.equal(out, t_in), "round trip differs"
    t0 = time.perf_counter()
    for _ in range(a.reps):
        comp.unlz4_device(fr.data_ptr(), size, out.data_ptr(), n)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.reps
    print(f"{a.shape} {n} B bs {bs}: frame {size} B, decode {dt * 1e3:.3f} ms = {n / dt / 1e9:.2f} GB/s, "
          f"reference chain hops {comp.unlz4_resolve_passes()}, round trip equal", flush=True)


if __name__ == "__main__":
    main()
