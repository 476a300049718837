#!/usr/bin/env python3
"""Diagnostic: k_unlz4_fix's serial re-joins on one bench shape's frame, from a SZ4_DIAG=8 build of the library
(tools/build_diag.sh 8): sub-segments, 64-wide batches, re-joins (and how many found nothing of the chain in
their sub-segment), tokens re-parsed, re-joins that met the speculative walk, clocks.
    python3 tools/diag_unlz4.py silesia|text4m"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SMALLZ4_AMD_LIB"] = os.path.join(ROOT, "smallz4_amd", "lib", "libsmallz4_amd_diag8.so")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import smallz4_amd  # noqa: E402
from prof_shape import SHAPES, shape_data  # noqa: E402


def main():
    shape = sys.argv[1] if len(sys.argv) > 1 else "silesia"
    full, bs, _ = SHAPES[shape]
    arr = shape_data(shape, full).copy()
    dev = torch.device("cuda:0")
    t_in = torch.from_numpy(arr).to(dev)
    comp = smallz4_amd.Compressor()
    lib = comp._lib
    lib.sz4_udiag_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    cap = lib.sz4_bound(full, bs)
    fr = torch.empty(cap, dtype=torch.uint8, device=dev)
    size = comp.compress_blocks_device(t_in.data_ptr(), full, fr.data_ptr(), cap, bs, 65535)
    out = torch.empty(full, dtype=torch.uint8, device=dev)
    comp.unlz4_device(fr.data_ptr(), size, out.data_ptr(), full)
    torch.cuda.synchronize()
    assert lib.sz4_udiag_clear() == 0
    comp.unlz4_device(fr.data_ptr(), size, out.data_ptr(), full)
    torch.cuda.synchronize()
    assert torch.equal(out, t_in)
    d = np.zeros(16, dtype=np.uint64)
    assert lib.sz4_udiag_read(d.ctypes.data, d.size) == 0
    nb = max(int(d[0]), 1)
    print(f"{shape}: blocks {int(d[0])}, sub-segments {int(d[1])}, batches {int(d[2])}, serial re-joins {int(d[3])} "
          f"(nothing of the chain in the sub-segment: {int(d[4])}; met the speculative walk: {int(d[6])}; most in one "
          f"block {int(d[10])}), tokens re-parsed {int(d[5])}")
    print(f"  clocks per block: mean {int(d[8]) / nb:.4g} (in re-joins {int(d[7]) / nb:.4g}), max {int(d[9])}")


if __name__ == "__main__":
    main()
