#!/usr/bin/env python3
"""A/B: the headline batch (100 MB, 64 KiB blocks, -9) as one call on one stream, against two halves
compressed at the same time by two contexts on two streams (two host threads; ctypes releases the GIL),
to see how much the chip gains from overlapping two pipelines."""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import smallz4_amd  # noqa: E402
from smallz4_amd import synth  # noqa: E402


def main():
    n = int(float(sys.argv[1]) * 1e6) if len(sys.argv) > 1 else 100_000_000
    reps = 10
    data = synth.enwik8_like(n, seed=8)
    dev = torch.device("cuda:0")
    t_in = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    cap = n + n // 8 + (1 << 20)
    outs = [torch.empty(cap, dtype=torch.uint8, device=dev) for _ in range(2)]
    comps = [smallz4_amd.Compressor(), smallz4_amd.Compressor()]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    half = (n // 2) // 65536 * 65536

    def one(k, lo, hi):
        comps[k].compress_blocks_device(t_in.data_ptr() + lo, hi - lo, outs[k].data_ptr(), cap, 65536, 65535, "none",
                                        streams[k].cuda_stream)

    for _ in range(2):
        one(0, 0, n)
        one(0, 0, half)
        one(1, half, n)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        one(0, 0, n)
    t1 = time.perf_counter()
    single = (t1 - t0) / reps
    t0 = time.perf_counter()
    for _ in range(reps):
        th = threading.Thread(target=one, args=(1, half, n))
        th.start()
        one(0, 0, half)
        th.join()
    t1 = time.perf_counter()
    pair = (t1 - t0) / reps
    t0 = time.perf_counter()
    for _ in range(reps):
        one(0, 0, half)
        one(1, half, n)
    t1 = time.perf_counter()
    seq = (t1 - t0) / reps
    print(f"single call {n / single / 1e6:.1f} MB/s ({single * 1e3:.3f} ms); two halves in turn "
          f"{n / seq / 1e6:.1f} MB/s ({seq * 1e3:.3f} ms); two halves at once {n / pair / 1e6:.1f} MB/s ({pair * 1e3:.3f} ms)")


if __name__ == "__main__":
    main()
