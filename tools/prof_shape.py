#!/usr/bin/env python3
"""Times one bench shape through sz4_compress_blocks_device (stage split, MB/s) -- short enough to run
under `rocprofv3 --kernel-trace --stats` or one `--pmc` pass per counter group.
    python3 tools/prof_shape.py silesia|text4m|zu|enwik8 [--mb MB] [--reps N] [--chain C]
The generated input is cached in /tmp (sz4_shape_<name>_<bytes>.bin) so that several passes over the
same shape generate it once.  SMALLZ4_AMD_LIB selects a variant build of the library."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import smallz4_amd  # noqa: E402
from smallz4_amd import synth  # noqa: E402

SHAPES = {
    "silesia": (211_938_580, 4 << 20, lambda n: synth.silesia_like(n, seed=2, workers=16)),
    "text4m": (100_000_000, 4 << 20, lambda n: synth.enwik8_like(n, seed=8)),
    "enwik8": (100_000_000, 65536, lambda n: synth.enwik8_like(n, seed=8)),
    "zu": ((10 << 30) // 8, 262144, lambda n: synth.zeros_urandom_range(0, n, seed=10)),
}


def shape_data(name, n):
    path = f"/tmp/sz4_shape_{name}_{n}.bin"
    if os.path.exists(path) and os.path.getsize(path) == n:
        return np.fromfile(path, dtype=np.uint8)
    data = SHAPES[name][2](n)
    arr = np.frombuffer(data, dtype=np.uint8)
    arr.tofile(path)
    return arr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("shape", choices=sorted(SHAPES))
    ap.add_argument("--mb", type=float, default=None)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--chain", type=int, default=65535)
    ap.add_argument("--stop-after", type=int, default=0,
                    help="sz4_debug_stop_after: 2 = after pass 1 (k_find_sorted); the SZ4_SKIP_* timing builds need it, "
                         "their wrong pass-1 results must not reach the later kernels")
    a = ap.parse_args()
    full, bs, _ = SHAPES[a.shape]
    n = int(a.mb * 1e6) if a.mb else full
    arr = shape_data(a.shape, n).copy()
    dev = torch.device("cuda:0")
    t_in = torch.from_numpy(arr).to(dev)
    comp = smallz4_amd.Compressor()
    cap = comp._lib.sz4_bound(n, bs)
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    comp.set_timing(True)
    if a.stop_after:
        comp.debug_stop_after(a.stop_after)
    comp.compress_blocks_device(t_in.data_ptr(), n, out.data_ptr(), cap, bs, a.chain)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st = {}
    for _ in range(a.reps):
        size = comp.compress_blocks_device(t_in.data_ptr(), n, out.data_ptr(), cap, bs, a.chain)
        for k, v in comp.last_stage_ms().items():
            st[k] = st.get(k, 0.0) + v / a.reps
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.reps
    print(f"{a.shape} {n} B bs {bs} chain {a.chain}: {n / dt / 1e6:.1f} MB/s ({dt * 1e3:.3f} ms), "
          f"ratio {size / n:.5f}, stages {({k: round(v, 3) for k, v in st.items()})}", flush=True)


if __name__ == "__main__":
    main()
