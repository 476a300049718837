#!/usr/bin/env python3
"""Diagnostic: k_find_big's phase clocks and counters from a SZ4_DIAG=6 build of the library
(tools/build_diag.sh 6 -> smallz4_amd/lib/libsmallz4_amd_diag6.so): workgroup-summed shader-clock ticks
per phase (group discovery, window load, run-group pieces / buckets / search, class path, the prefix
maximum) on a Silesia-shaped input at 4 MiB blocks, -9."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SMALLZ4_AMD_LIB"] = os.path.join(ROOT, "smallz4_amd", "lib", "libsmallz4_amd_diag6.so")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import smallz4_amd  # noqa: E402
from smallz4_amd import synth  # noqa: E402


def main():
    mb = float(sys.argv[1]) if len(sys.argv) > 1 else 64
    workload = sys.argv[2] if len(sys.argv) > 2 else "silesia"
    n = int(mb * 1e6)
    if workload == "zu":  # configs[4]: zeros/urandom at 256 KiB blocks
        data, bs = synth.zeros_urandom_range(0, n, seed=10), 262144
    else:
        data, bs = synth.silesia_like(n, workers=8), 4 << 20
    comp = smallz4_amd.Compressor()
    lib = comp._lib
    lib.sz4_diag_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    comp.compress_blocks(data, bs, 65535)
    assert lib.sz4_diag_clear() == 0
    comp.set_timing(True)
    comp.compress_blocks(data, bs, 65535)
    st = comp.last_stage_ms()
    buf = np.zeros(32, dtype=np.uint64)
    assert lib.sz4_diag_read(buf.ctypes.data, buf.size) == 0
    names = {0: "groups found", 1: "window load", 6: "run group: entry", 2: "run group: pieces", 3: "run group: buckets",
             5: "run group: search", 7: "class path", 4: "after the groups"}
    tot = sum(int(buf[k]) for k in names)
    print(f"{mb:.0f} MB {workload}, {bs >> 10} KiB blocks, -9: stages {st}")
    for k, name in names.items():
        print(f"  tick[{k}] {name:22s} {int(buf[k]):.4g} ({100.0 * int(buf[k]) / max(tot, 1):.1f} %)")
    cnt = {8: "run targets", 9: "same-R piece visits", 10: "c10", 11: "c11", 12: "pieces", 13: "class groups",
           14: "run groups", 15: "segments (first launch)", 16: "bad pieces", 17: "mixed run groups",
           18: "too many pieces", 19: "c19", 20: "c20", 21: "wave ticks 21", 22: "wave ticks 22", 23: "wave ticks 23",
           24: "no big group", 25: "too many groups", 26: "c26", 27: "c27"}
    print("  " + ", ".join(f"{v} {int(buf[k])}" for k, v in cnt.items()))


if __name__ == "__main__":
    main()
