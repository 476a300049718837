#!/usr/bin/env python3
"""Diagnostic: k_dp_fix<false>'s serial repair on configs[4]'s input (zeros/urandom, 256 KiB blocks, -9) from
a SZ4_DIAG=7 build of the library (tools/build_diag.sh 7): positions repaired one at a time, closed-form and
literal chunks, segments walked, per-block clock (sum and max)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SMALLZ4_AMD_LIB"] = os.path.join(ROOT, "smallz4_amd", "lib", "libsmallz4_amd_diag7.so")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import smallz4_amd  # noqa: E402
from smallz4_amd import synth  # noqa: E402


def main():
    mb = float(sys.argv[1]) if len(sys.argv) > 1 else 256
    n = int(mb * (1 << 20))
    data = synth.zeros_urandom_range(0, n, seed=10)
    comp = smallz4_amd.Compressor()
    lib = comp._lib
    lib.sz4_diag_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    comp.compress_blocks(data, 262144, 65535)
    assert lib.sz4_diag_clear() == 0
    comp.set_timing(True)
    comp.compress_blocks(data, 262144, 65535)
    st = comp.last_stage_ms()
    d = np.zeros(16, dtype=np.uint64)
    assert lib.sz4_diag_read(d.ctypes.data, d.size) == 0
    nb = int(d[7])
    print(f"{mb:g} MiB zeros/urandom, 256 KiB blocks, -9: stages {st}")
    print(f"  blocks {nb} (rmq {int(d[8])}), segments walked {int(d[3])}, serial positions {int(d[0])} "
          f"(max per block {int(d[4])}), closed chunks {int(d[1])}, literal chunks {int(d[2])}")
    print(f"  ticks per block: mean {int(d[5]) / max(nb, 1):.4g}, max {int(d[6])}")
    tk = [int(x) for x in d[9:13]]
    print("  ticks by chunk kind (sum over blocks): " + ", ".join(
        f"{k} {v:.4g} ({100 * v / max(int(d[5]), 1):.1f} %)" for k, v in zip(("literal", "closed", "serial", "rmq stores"), tk)))


if __name__ == "__main__":
    main()
