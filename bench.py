#!/usr/bin/env python3
"""bench.py -- BASELINE.json's metric on MI355X.

metric : input MB/s at -9 optimal parse; output-byte diff vs smallz4 (must be 0)
workload (BASELINE configs[1]): enwik8-shaped input (100 MB per GPU, synthetic --
    enwik8 itself is not available offline) compressed as independent 64 KiB
    blocks at -9 (maxChainLength 65535).  One step = one full compression of the
    rank's 100 MB, input resident in HBM, frame written to HBM.
multi-GPU: one process per GPU; blocks shard with no data-path collective
    (weak scaling: every rank compresses its own 100 MB).  The barrier and the
    max-over-ranks timing are the only collectives.

Also reported:
  byte_diff     differing bytes between the GPU frame and the reference's output for
                every block (oracle/_ref, compiled from the reference sources; the C
                restatement when _ref is absent), all blocks, every rank
  roofline      dominant kernel (k_find_sorted), HIP-event timed on its stream
  cpu_baseline  the reference itself on this host, one thread, bounded sample
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from smallz4_amd import synth  # noqa: E402  (input generators; the HIP library loads lazily)

METRIC = "input MB/s at -9 optimal parse; output-byte diff vs smallz4 (must be 0)"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
PMC_FILE = os.path.join(ROOT, "profiles", "r01h_find_hbm_bytes.json")  # k_find_sorted HBM bytes (summarize.py)

# input shapes (smallz4_amd/synth.py); the default is the headline workload (configs[1])
DATA = {
    "enwik8": ("synthetic enwik8-shaped text (smallz4_amd/synth.py; enwik8 is not available offline)",
               lambda n, seed: synth.enwik8_like(n, seed=seed)),
    "zeros_urandom": ("synthetic: alternating 128 KiB runs of zeros and urandom bytes (configs[4]'s two extremes)",
                      lambda n, seed: synth.zeros_urandom(n, seed=seed)),
    "zeros": ("synthetic: all zero bytes", lambda n, seed: bytes(n)),
    "random": ("synthetic: urandom bytes (numpy, seeded)", lambda n, seed: synth.random_bytes(n, seed=seed)),
}


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mb", type=float, default=100.0, help="input MB (1e6 bytes) per GPU")
    ap.add_argument("--block-size", type=int, default=65536)
    ap.add_argument("--level", type=int, default=9)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    ap.add_argument("--verify-threads", type=int, default=16)
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-decode", action="store_true", help="skip the decoder leg (sz4_unlz4_device)")
    ap.add_argument("--data", default="enwik8", choices=sorted(DATA),
                    help="synthetic input shape (enwik8: configs[1]; zeros_urandom: configs[4])")
    return ap.parse_args()


def expected_blocks(data: bytes, bs: int, chain: int, threads: int):
    """Per-block reference output (block word + payload), computed on the CPU."""
    from oracle import pyoracle
    if pyoracle.ref_available():
        def one(off):
            f = pyoracle.ref_lz4(data[off:off + bs], chain)
            return f[7:-4]
        kind = "reference"
    else:
        def one(off):
            return pyoracle.oz_block(data[off:off + bs], chain)
        kind = "port"
    with ThreadPoolExecutor(max_workers=threads) as ex:
        parts = list(ex.map(one, range(0, len(data), bs)))
    return parts, kind


def byte_diff(frame: bytes, parts, header: bytes) -> int:
    expect = header + b"".join(parts) + b"\0\0\0\0"
    n = min(len(frame), len(expect))
    import numpy as np
    a = np.frombuffer(frame[:n], dtype=np.uint8)
    b = np.frombuffer(expect[:n], dtype=np.uint8)
    return int((a != b).sum()) + abs(len(frame) - len(expect))


def cpu_baseline(data: bytes, bs: int, chain: int, budget_s: float):
    from oracle import pyoracle
    if pyoracle.ref_available():
        fn, kind = (lambda b: pyoracle.ref_lz4(b, chain)), "reference"
    else:
        fn, kind = (lambda b: pyoracle.oz_block(b, chain)), "port"
    done = 0
    t0 = time.perf_counter()
    for off in range(0, len(data), bs):
        fn(data[off:off + bs])
        done += min(bs, len(data) - off)
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": round(done / dt / 1e6, 3), "unit": "MB/s", "cores": 1, "kind": kind,
            "sample": f"first {done / 1e6:.1f} MB of the rank-0 input as {bs}-byte blocks, level chain={chain}, "
                      f"one thread, smallz4::lz4 per block ({dt:.1f} s)"}


def main():
    args = parse_args()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)

    import smallz4_amd

    chain = smallz4_amd.level_to_chain(args.level)
    nbytes = int(args.mb * 1e6)
    data = DATA[args.data][1](nbytes, 8 + rank)
    t_in = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda(local)
    comp = smallz4_amd.Compressor(device=local)
    cap = comp._lib.sz4_bound(nbytes, args.block_size)
    out = torch.empty(cap, dtype=torch.uint8, device=f"cuda:{local}")
    stream = torch.cuda.current_stream(local).cuda_stream

    def step():
        return comp.compress_blocks_device(t_in.data_ptr(), nbytes, out.data_ptr(), cap, args.block_size, chain,
                                           "smallz4", stream)

    comp.set_timing(True)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(local)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(local)
    t0 = time.perf_counter()
    stage_sum = {}
    size = 0
    for _ in range(args.steps):
        size = step()
        for k, v in comp.last_stage_ms().items():
            stage_sum[k] = stage_sum.get(k, 0.0) + v
    torch.cuda.synchronize(local)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(local)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    stages = {k: v / args.steps for k, v in stage_sum.items()}
    frame = out[:size].cpu().numpy().tobytes()

    # decoder leg (smallz4cat semantics on the device, sz4_unlz4_device), outside the timed region:
    # the frame just written, decoded back into HBM and compared with the input
    dec = None
    if not args.no_decode:
        dout = torch.empty(nbytes, dtype=torch.uint8, device=f"cuda:{local}")
        comp.unlz4_device(out.data_ptr(), size, dout.data_ptr(), nbytes, stream=stream)
        torch.cuda.synchronize(local)
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            got = comp.unlz4_device(out.data_ptr(), size, dout.data_ptr(), nbytes, stream=stream)
        torch.cuda.synchronize(local)
        dt = (time.perf_counter() - t0) / reps
        dec = {"value": round(nbytes / dt / 1e6, 1), "unit": "MB/s of decoded output (host-timed call: index, "
               "sizes and decode launches with their syncs)", "ms": round(dt * 1e3, 3),
               "roundtrip_equal": bool(got == nbytes and torch.equal(dout, t_in))}
        del dout

    # output-byte diff against the reference, every block of every rank
    diff, verified, kind = -1, 0, None
    if not args.no_verify:
        parts, kind = expected_blocks(data, args.block_size, chain, args.verify_threads)
        diff = byte_diff(frame, parts, bytes([0x04, 0x22, 0x4D, 0x18, 0x40, 0x70, 0xDF]))
        verified = len(parts)
        if world > 1:
            t = torch.tensor([diff, verified], dtype=torch.int64, device=f"cuda:{local}")
            dist.all_reduce(t)
            diff, verified = int(t[0]), int(t[1])

    if rank == 0:
        value = world * nbytes * args.steps / elapsed / 1e6
        # roofline of the dominant kernel k_find_sorted.  Its compulsory HBM bytes
        # per position: text byte (1) + sorted slot arrays, u16 position and group start (4, read; with
        # the sort fused in, written) + match, u32 length and u16 distance (6, written); fused, also
        # the rank of every target (4, written)
        fused = os.environ.get("SZ4_SEPARATE_SORT", "") != "1"
        find_ms = stages.get("find_sorted", 0.0)
        targets = sum(max(0, min(args.block_size, nbytes - o) - 11) for o in range(0, nbytes, args.block_size))
        alg_bytes = nbytes + 4 * nbytes + 6 * targets + (4 * targets if fused else 0)
        achieved = alg_bytes / (find_ms * 1e-3) / 1e9 if find_ms > 0 else 0.0
        traffic = None
        default_cfg = args.data == "enwik8" and args.block_size == 65536 and args.level == 9 and nbytes == 100_000_000
        if default_cfg and fused and os.path.exists(PMC_FILE):
            with open(PMC_FILE) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        kname = "k_find_sorted (k_sort fused in)" if fused else "k_find_sorted"
        rec = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "MB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": DATA[args.data][0],
            "config": {"workload": f"{args.data}-shaped {args.mb:g} MB per GPU as independent {args.block_size}-byte "
                                   f"blocks, level -{args.level} (maxChainLength {chain})",
                       "block_size": args.block_size, "level": args.level, "bytes_per_gpu": nbytes,
                       "parallelism": f"blocks sharded over {world} GPU(s), no data-path collective"},
            "byte_diff": diff,
            "blocks_verified": verified,
            "verified_against": kind,
            "compression_ratio": round(size / nbytes, 5),
            "stages_ms": {k: round(v, 3) for k, v in stages.items()},
            "roofline": {"kernel": kname, "bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
                         "algorithmic_bytes_per_launch": alg_bytes},
        }
        if dec is not None:
            rec["unlz4"] = dec
        if world == 1:
            rec["cpu_baseline"] = cpu_baseline(data, args.block_size, chain, args.cpu_seconds)
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
