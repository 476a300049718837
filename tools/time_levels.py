#!/usr/bin/env python3
"""Times configs[1]'s input (100 MB, 64 KiB blocks) at the given reference levels (maxChainLength per
smallz4.cpp:232-238: -N -> N for N <= 8, -9 -> 65535) with the stage split; run under
`rocprofv3 --kernel-trace --stats` for the per-kernel picture.
    python3 tools/time_levels.py 3 6 [--mb 100]"""
import argparse
import hashlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import smallz4_amd  # noqa: E402
from smallz4_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("levels", nargs="+", type=int)
    ap.add_argument("--mb", type=float, default=100)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    n = int(a.mb * 1e6)
    data = synth.enwik8_like(n, seed=8)
    dev = torch.device("cuda:0")
    t_in = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    cap = n + n // 8 + (1 << 20)
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    comp = smallz4_amd.Compressor()
    comp.set_timing(True)
    for lv in a.levels:
        chain = 65535 if lv >= 9 else lv
        comp.compress_blocks_device(t_in.data_ptr(), n, out.data_ptr(), cap, 65536, chain)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            size = comp.compress_blocks_device(t_in.data_ptr(), n, out.data_ptr(), cap, 65536, chain)
        dt = (time.perf_counter() - t0) / a.reps
        st = {k: round(v, 3) for k, v in comp.last_stage_ms().items()}
        sha = hashlib.sha256(out[:size].cpu().numpy().tobytes()).hexdigest()[:16]
        print(f"-{lv}: {n / dt / 1e6:.1f} MB/s ({dt * 1e3:.3f} ms), ratio {size / n:.4f}, frame {sha}, stages {st}",
              flush=True)


if __name__ == "__main__":
    main()
