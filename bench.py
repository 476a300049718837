#!/usr/bin/env python3
"""bench.py -- BASELINE.json's metric on MI355X.

metric : input MB/s at -9 optimal parse; output-byte diff vs smallz4 (must be 0)

workloads (BASELINE.json configs; all synthetic, the corpora are not available offline):
  enwik8        configs[1]: 100 MB enwik8-shaped text, independent 64 KiB blocks, -9.  The default at
                N=1 (the configuration the metric is quoted on).
  enwik9        configs[3]: an enwik9-shaped input (10^9 bytes at 8 GPUs) in 64 KiB blocks, sharded:
                rank r of N compresses its contiguous block range of the first N x 125 MB, so every
                GPU does the same work at any N (weak scaling) and N=8 is the whole 10^9 bytes.  The
                default at N>1; at N=1 the `shapes` leg measures the same 125 MB per GPU, so a 1->8
                curve can be read on one workload.
  zeros_urandom configs[4]: 10 GiB of zero and urandom runs of random lengths (mean 128 KiB, 50/50
                bytes, runs straddling the block grid) at 8 GPUs, 256 KiB blocks, sharded the same way
                (1.25 GiB per GPU).
  silesia       configs[2]: Silesia-shaped mixed content (text, XML, executables, database rows,
                images, source), 4 MiB independent blocks, 1 GPU.
One step = one full compression of the rank's shard, input resident in HBM, blocks written to HBM.

multi-GPU: one process per GPU.  Blocks are independent, so ranks shard the block range of ONE input
(smallz4_amd/shard.py) with no data-path collective; each rank's part (bare blocks; rank 0 adds the
header, the last rank the end mark) concatenates to the single-GPU frame.  The barrier, the
max-over-ranks time and the result reductions are the only collectives.  `--gpus N` without a
torch.distributed environment starts N ranks itself (a torch.distributed.run child process, before
this process touches the GPU) and exits with its status.

Also reported:
  byte_diff      differing bytes between the GPU blocks and the reference's output for the same
                 blocks (oracle/_ref/smallz4, the reference CLI compiled from its sources, one child
                 process per block with a hard deadline; the C restatement when _ref is absent):
                 every block at N=1 on enwik8, otherwise a seeded random sample bounded by
                 --verify-seconds
  roundtrip      every rank's part decoded on the device (sz4_unlz4_device) equals its input
  roofline       dominant kernel (k_find_sorted), HIP-event timed on its stream; HBM traffic from the
                 newest matching profiles/*_pmc.json (rocprofv3 PMC passes of the same workload)
  cpu_baseline   the reference itself on this host (rank 0, every N, after the timed region): one
                 thread per CPU this process may use (affinity mask, capped by the cgroup quota; the
                 count is recorded), and one thread, on a bounded sample
  stream         the C++ drop-in (smallz4::lz4 through include/smallz4_amd.hpp, tools/bin/stream_threads):
                 1 GB, 4 MiB dependent blocks in 64 MiB chunks, callbacks and PCIe in the clock, its own
                 device footprint; N=1, outside the timed region
  dictionary     sz4_lz4 with a 64 KiB dictionary: 8 MB at -9 and -6 diffed against the reference, and
                 8 MB with a 200 KB zero run (the same-letter shortcut) against the reference's frame hash
  shapes         N=1: the other single-GPU-sized configs -- configs[2] (Silesia-shaped, 4 MiB blocks),
                 configs[4]'s 1.25 GiB rank slice, text at 4 MiB blocks, configs[3]'s 125 MB rank slice
                 -- each with ms/step, MB/s, a sampled byte_diff bounded by seconds, and the round trip
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import re
import subprocess
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from smallz4_amd import shard, synth  # noqa: E402  (input generators; the HIP library loads lazily)

METRIC = "input MB/s at -9 optimal parse; output-byte diff vs smallz4 (must be 0)"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec
CLOCK_GHZ = 2.4         # MI355X_MICROARCH.md: max clock
SIMDS, CUS = 1024, 256  # 256 CUs x 4 SIMDs


def host_cpus():
    """(threads the CPU baseline runs on, how they were found): the CPUs this process may run on
    (sched_getaffinity), lowered to the cgroup CPU quota when one is set (cpu.max: a quota limits
    throughput without shrinking the affinity mask)."""
    n = len(os.sched_getaffinity(0))
    src = f"sched_getaffinity: {n}"
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            q = max(1, int(-(-int(quota) // int(period))))
            src += f", cgroup cpu.max quota: {q}"
            n = min(n, q)
    except (OSError, ValueError):
        pass
    return n, src


HOST_THREADS, HOST_THREADS_SOURCE = host_cpus()
POOL = min(HOST_THREADS, 16)  # generator processes and reference-diff workers (the box's share per GPU)

# name -> (BASELINE config, description, block size, bytes per rank at N ranks, range generator)
WORKLOADS = {
    "enwik8": ("configs[1]", "synthetic enwik8-shaped text (smallz4_amd/synth.py; enwik8 is not available offline)",
               65536, lambda world: 100_000_000,
               lambda lo, hi: synth.enwik8_like(100_000_000, seed=8)[lo:hi]),
    "enwik9": ("configs[3]", "synthetic enwik9-shaped text: 16 MiB enwik8-shaped segments (synth.enwik9_like_range)",
               65536, lambda world: 125_000_000,
               lambda lo, hi: synth.enwik9_like_range(lo, hi, seed=9, workers=POOL)),
    "zeros_urandom": ("configs[4]", "synthetic: zero and urandom runs of random lengths, mean 128 KiB, 50/50 bytes "
                                    "(synth.zeros_urandom_range)",
                      262144, lambda world: (10 << 30) // 8,
                      lambda lo, hi: synth.zeros_urandom_range(lo, hi, seed=10)),
    "silesia": ("configs[2]", "synthetic Silesia-shaped mixed content (synth.silesia_like; the corpus is not available offline)",
                4 << 20, lambda world: 211_938_580,
                lambda lo, hi: synth.silesia_like(hi, seed=2, workers=POOL)[lo:hi]),
    # diagnostic shapes (not BASELINE configs): the kernels' floors on incompressible / all-run data
    "random": ("diagnostic", "synthetic: urandom bytes (numpy, seeded)", 65536, lambda world: 100_000_000,
               lambda lo, hi: synth.random_bytes(hi, seed=8)[lo:hi]),
    "zeros": ("diagnostic", "synthetic: all zero bytes", 65536, lambda world: 100_000_000,
              lambda lo, hi: bytes(hi - lo)),
}

# the shapes leg at N=1: (label, workload, block size override)
SHAPES = [("silesia_4m", "silesia", None), ("zeros_urandom_256k", "zeros_urandom", None),
          ("enwik8_4m", "enwik8", 4 << 20), ("enwik9_rank_slice", "enwik9", None)]


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default=None,
                    help="default: enwik8 (configs[1]) at one GPU, enwik9 (configs[3]) at several")
    ap.add_argument("--mb", type=float, default=None, help="override: input MB (1e6 bytes) per rank")
    ap.add_argument("--block-size", type=int, default=None, help="override the workload's block size")
    ap.add_argument("--level", type=int, default=9)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="budget of each CPU baseline sample")
    ap.add_argument("--verify-threads", type=int, default=POOL)
    ap.add_argument("--verify-seconds", type=float, default=20.0,
                    help="per-rank budget of the sampled byte diff against the reference (the whole "
                         "input at N=1 on enwik8 is always diffed)")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-decode", action="store_true", help="skip the device round trip (sz4_unlz4_device)")
    ap.add_argument("--no-stream", action="store_true", help="skip the C++ drop-in stream leg")
    ap.add_argument("--stream-reps", type=int, default=10, help="stream leg: 100 MB repetitions (10 = 1 GB)")
    ap.add_argument("--no-dict", action="store_true", help="skip the dictionary-mode leg")
    ap.add_argument("--no-shapes", action="store_true", help="skip the other configs (N=1)")
    ap.add_argument("--no-levels", action="store_true", help="skip the levels leg (-1, -3, -6, -8 on configs[1])")
    ap.add_argument("--level-steps", type=int, default=3)
    ap.add_argument("--level-verify-seconds", type=float, default=6.0)
    ap.add_argument("--level-cpu-seconds", type=float, default=3.0, help="levels leg: budget of each CPU baseline sample")
    ap.add_argument("--shape-steps", type=int, default=3)
    ap.add_argument("--shape-verify-seconds", type=float, default=8.0)
    ap.add_argument("--silesia-verify-seconds", type=float, default=150.0,
                    help="configs[2]'s diff budget: enough for all 51 blocks (the reference takes 10-60 s per 4 MiB block)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: gloo ranks compress their shards with the oracle (tests the sharding)")
    a = ap.parse_args(argv)
    if a.workload is None:
        a.workload = "enwik8" if a.gpus == 1 else "enwik9"
    return a


def rank_range(args, world, rank, workload=None, block_size=None, mb=None):
    """(global input length, [lo, hi) of this rank, block size)."""
    wl = WORKLOADS[workload or args.workload]
    bs = block_size or args.block_size or wl[2]
    mb = mb if mb is not None else args.mb
    per = int(mb * 1e6) if mb else wl[3](world)
    total = per * world
    lo, hi = shard.shard_range(total, bs, rank, world)
    return total, lo, hi, bs


def block_spans(part: bytes):
    """(offset, length) of every block (word + payload) in a run of bare blocks."""
    spans, pos = [], 0
    while pos + 4 <= len(part):
        word = int.from_bytes(part[pos:pos + 4], "little")
        n = 4 + (word & 0x7FFFFFFF)
        spans.append((pos, n))
        pos += n
    return spans


def _level_flag(chain: int) -> str:
    return "-9" if chain >= 65535 else f"-{chain}"


def verify_sample(part: bytes, data: bytes, bs: int, chain: int, threads: int, budget_s: float, every: bool):
    """Byte diff of this rank's blocks against the reference.  Blocks are taken in a seeded random
    order (all of them when `every`), each compressed by the reference CLI (oracle/_ref/smallz4) in a
    child process that is killed at the deadline, so the leg is bounded by `budget_s` whatever one
    block costs the reference (4 MiB of binary records: ~2 minutes at -9)."""
    import numpy as np
    from oracle import pyoracle
    spans = block_spans(part)
    nblk = (len(data) + bs - 1) // bs
    if len(spans) != nblk:
        return {"byte_diff": len(part) + 1, "blocks_verified": 0, "blocks_total": nblk, "verified_against": None,
                "note": "block count differs"}
    order = list(range(nblk)) if every else [int(i) for i in np.random.default_rng(2024).permutation(nblk)]
    cli = os.path.join(ROOT, "oracle", "_ref", "smallz4")
    use_cli = os.path.exists(cli)
    kind = "reference" if use_cli else "port"
    t0 = time.perf_counter()
    deadline = t0 + budget_s

    def one(i):
        block = data[i * bs:(i + 1) * bs]
        left = deadline - time.perf_counter()
        if left <= 0.05:
            return i, None
        if use_cli:
            try:
                r = subprocess.run([cli, _level_flag(chain), "-f"], input=block, capture_output=True, timeout=left)
            except subprocess.TimeoutExpired:
                return i, None
            if r.returncode != 0:
                return i, b""
            return i, r.stdout[7:-4]
        return i, pyoracle.oz_block(block, chain)

    diff, done = 0, 0
    with ThreadPoolExecutor(max_workers=threads) as ex:
        for i, want in ex.map(one, order):
            if want is None:
                continue
            o, n = spans[i]
            got = part[o:o + n]
            if got != want:
                m = min(len(got), len(want))
                diff += sum(1 for a, b in zip(got[:m], want[:m]) if a != b) + abs(len(got) - len(want))
            done += 1
    complete = done == nblk
    if every and not complete:
        sample = f"every block requested, {nblk - done} not diffed (reference timeout or budget): incomplete"
    elif every:
        sample = "every block"
    else:
        sample = "seeded random order, cut at the budget"
    return {"byte_diff": diff if (complete or not every) else -1, "byte_diff_of_verified": diff,
            "blocks_verified": done, "blocks_total": nblk, "verified_against": kind, "verify_complete": complete,
            "verify_seconds": round(time.perf_counter() - t0, 2), "verify_budget_s": budget_s,
            "verify_sample": sample}


def cpu_baseline(data: bytes, bs: int, chain: int, budget_s: float):
    """The reference (oracle/_ref; the C restatement when absent) on a bounded sample, all threads
    of the box's share and one thread."""
    from oracle import pyoracle
    if pyoracle.ref_available():
        fn, kind = (lambda b: pyoracle.ref_lz4(b, chain)), "reference"
    else:
        fn, kind = (lambda b: pyoracle.oz_block(b, chain)), "port"
    offs = list(range(0, len(data), bs))

    def run(threads):
        done, t0 = 0, time.perf_counter()
        with ThreadPoolExecutor(max_workers=threads) as ex:
            k = 0
            while k < len(offs) and time.perf_counter() - t0 < budget_s:
                batch = offs[k:k + threads]
                for b in ex.map(lambda o: fn(data[o:o + bs]), batch):
                    pass
                done += sum(min(bs, len(data) - o) for o in batch)
                k += len(batch)
        return done, time.perf_counter() - t0

    done_n, dt_n = run(HOST_THREADS)
    done_1, dt_1 = run(1)
    return {"value": round(done_n / dt_n / 1e6, 3), "unit": "MB/s", "cores": HOST_THREADS,
            "cores_source": HOST_THREADS_SOURCE, "kind": kind,
            "sample": f"first {done_n / 1e6:.1f} MB of the rank-0 shard as {bs}-byte blocks, maxChainLength {chain}, "
                      f"smallz4::lz4 per block on {HOST_THREADS} threads ({dt_n:.1f} s)",
            "single_thread": {"value": round(done_1 / dt_1 / 1e6, 3), "cores": 1,
                              "sample": f"first {done_1 / 1e6:.1f} MB, one thread ({dt_1:.1f} s)"}}


def pmc_tag_key(tag: str):
    """Order of profile tags rNN<suffix>: round, suffix length, suffix."""
    m = re.match(r"r(\d+)([a-z]*)$", tag)
    return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, len(tag), tag)


def pmc_traffic(cfg):
    """HBM bytes per k_find_sorted launch from the newest profiles/**/*_pmc.json of this workload."""
    best = None
    # tags run r02a..r02z, r02aa..r02az, then r03a..: order by round, then suffix length, then suffix
    # (so r02av sorts after r02o, and r03a after r02bd)
    paths = glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")) + \
        glob.glob(os.path.join(ROOT, "profiles", "*", "*_pmc.json"))
    for path in sorted(paths, key=lambda p: pmc_tag_key(os.path.basename(p)[: -len("_pmc.json")])):
        try:
            with open(path) as f:
                rec = json.load(f)
        except (OSError, ValueError):
            continue
        if rec.get("config") == cfg:
            best = (path, rec)
    return best


def valu_ceiling():
    """The integer VALU issue rate the MI355X sustains (tools/valu_ceiling.hip, every SIMD at 8 waves,
    independent add/xor chains, the clock read in the same run from s_memtime against s_memrealtime), from
    the newest profiles/valu_ceiling_*.json: {"source", "vgpr": per SIMD-cycle at its measured clock with
    VGPR operands (the shift-register and DPP tests), "sgpr": the same with SGPR operands (readlane
    broadcasts), "clock_ghz"}.  Round 4's record (no clock, one variant) is read at CLOCK_GHZ."""
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "valu_ceiling_*.json")))
    if not paths:
        return None
    recs = []
    with open(paths[-1]) as f:
        for line in f:
            try:
                recs.append(json.loads(line))
            except ValueError:
                continue
    out = {"source": os.path.relpath(paths[-1], ROOT)}
    full = [r for r in recs if r.get("waves_per_simd") == 8 and "per_simd_per_cycle" in r]
    if full:
        vg = [r for r in full if "vgpr" in r["variant"] or "4chains" in r["variant"]]
        sg = [r for r in full if r["variant"] in ("add_xor_8chains", "add_16chains")]
        if vg:
            best = max(vg, key=lambda r: r["per_simd_per_cycle"])
            out.update({"vgpr": best["per_simd_per_cycle"], "clock_ghz": best["clock_ghz_median"], "variant": best["variant"]})
        if sg:
            out["sgpr"] = max(r["per_simd_per_cycle"] for r in sg)
        return out if "vgpr" in out else None
    best = max((r["valu_instr_per_s"] for r in recs if r.get("variant") == "add_xor"), default=0.0)
    if not best:
        return None
    out.update({"vgpr": round(best / 1024 / (CLOCK_GHZ * 1e9), 4), "clock_ghz": CLOCK_GHZ, "variant": "add_xor"})
    return out


def summary_line(rec) -> str:
    """A short plain-text recap printed after the JSON line (not JSON, so nothing parses it as the
    record): the headline's own parity and roofline, and each shape's rate and diff, where a log tail
    that cuts the long line still shows them."""
    ver = rec.get("verify", {})
    parts = [f"summary: value {rec['value']} MB/s", f"byte_diff {rec['byte_diff']}",
             f"blocks_verified {rec['blocks_verified']}/{ver.get('blocks_total', '?')}",
             f"roundtrip_ok {rec['roundtrip_ok']}", f"roofline.frac {rec['roofline']['frac']}"]
    for label, sh in (rec.get("shapes") or {}).items():
        parts.append(f"{label} {sh['MB/s']} MB/s byte_diff {sh.get('byte_diff')} "
                     f"({sh.get('blocks_verified')}/{sh.get('blocks_total')} blocks, verify_complete {sh.get('verify_complete')})")
    for lv, r in ((rec.get("levels") or {}).get("levels") or {}).items():
        parts.append(f"level {lv} {r['MB/s']} MB/s byte_diff {r.get('byte_diff')}")
    return "; ".join(parts)


def spawn_ranks(args):
    """`--gpus N` outside torch.distributed: run N ranks through torch.distributed.run as a child
    process (this process has not touched the GPU) and return its exit status."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.call(cmd, env=env)


def dry_run(args, world, rank):
    """HIP-free rehearsal of the sharded path (gloo): each rank compresses its block range with the
    oracle; rank 0 checks that the parts concatenate to the single-process frame, and reports the
    fields the GPU line would carry (workload, cpu_baseline, verify budget)."""
    import torch.distributed as dist
    from oracle import pyoracle
    if world > 1:
        dist.init_process_group("gloo")
    total, lo, hi, bs = rank_range(args, world, rank)
    data = WORKLOADS[args.workload][4](lo, hi)
    chain = 65535 if args.level == 9 else args.level
    body = b"".join(pyoracle.oz_block(data[o:o + bs], chain) for o in range(0, len(data), bs))
    part = shard.frame_part(body, rank, world)
    frame = shard.gather_frame(part) if world > 1 else part
    if rank == 0:
        whole = WORKLOADS[args.workload][4](0, total)
        single = shard.HEADER + b"".join(pyoracle.oz_block(whole[o:o + bs], chain)
                                         for o in range(0, total, bs)) + shard.END_MARK
        rec = {"dry_run": True, "n_gpus": world, "workload": args.workload, "input_bytes": total,
               "bytes_per_gpu": hi - lo, "frame_bytes": len(frame), "parts_equal_single": frame == single,
               "verify_budget_s": args.verify_seconds,
               "cpu_baseline": cpu_baseline(data, bs, chain, min(args.cpu_seconds, 0.5))}
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


class Runner:
    """One rank's GPU state: the compressor context, its device and stream."""

    def __init__(self, local):
        import torch
        import smallz4_amd
        self.torch = torch
        self.local = local
        self.dev = f"cuda:{local}"
        self.comp = smallz4_amd.Compressor(device=local)
        self.stream = torch.cuda.current_stream(local).cuda_stream

    def compress(self, data: bytes, bs: int, chain: int, steps: int, warmup: int, header: str, barrier=None):
        """Timed compression of `data` (resident in HBM): (seconds of `steps` steps, mean stage ms,
        frame bytes, the frame tensor, the input tensor)."""
        torch = self.torch
        n = len(data)
        t_in = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(self.dev) if n else \
            torch.empty(0, dtype=torch.uint8, device=self.dev)
        cap = self.comp._lib.sz4_bound(n, bs)
        out = torch.empty(max(cap, 16), dtype=torch.uint8, device=self.dev)

        def step():
            return self.comp.compress_blocks_device(t_in.data_ptr() if n else out.data_ptr(), n, out.data_ptr(), cap,
                                                    bs, chain, header, self.stream)

        self.comp.set_timing(True)
        for _ in range(warmup):
            step()
        torch.cuda.synchronize(self.local)
        if barrier:
            barrier()
        torch.cuda.synchronize(self.local)
        t0 = time.perf_counter()
        stage_sum, size = {}, 0
        for _ in range(steps):
            size = step()
            for k, v in self.comp.last_stage_ms().items():
                stage_sum[k] = stage_sum.get(k, 0.0) + v
        torch.cuda.synchronize(self.local)
        if barrier:
            barrier()
        torch.cuda.synchronize(self.local)
        elapsed = time.perf_counter() - t0
        return elapsed, {k: v / max(steps, 1) for k, v in stage_sum.items()}, size, out, t_in

    def roundtrip(self, out, size: int, header: str, t_in, reps: int = 3):
        """Decode this rank's blocks on the device (sz4_unlz4_device): (equal to the input, timing)."""
        torch = self.torch
        n = t_in.numel()
        if not n:
            return True, None
        off = 7 if header == "smallz4" else 0
        nbody = size - off - (4 if header == "smallz4" else 0)
        fr = torch.empty(nbody + 11, dtype=torch.uint8, device=self.dev)
        fr[:7] = torch.tensor(list(shard.HEADER), dtype=torch.uint8)
        fr[7:7 + nbody] = out[off:off + nbody]
        fr[7 + nbody:] = 0
        dout = torch.empty(n, dtype=torch.uint8, device=self.dev)
        self.comp.unlz4_device(fr.data_ptr(), fr.numel(), dout.data_ptr(), n, stream=self.stream)
        torch.cuda.synchronize(self.local)
        td = time.perf_counter()
        got = 0
        for _ in range(reps):
            got = self.comp.unlz4_device(fr.data_ptr(), fr.numel(), dout.data_ptr(), n, stream=self.stream)
        torch.cuda.synchronize(self.local)
        dt = (time.perf_counter() - td) / reps
        ok = bool(got == n and torch.equal(dout, t_in))
        del dout, fr
        return ok, {"value": round(n / dt / 1e6, 1), "unit": "MB/s of decoded output (host-timed call: index, sizes "
                    "and decode launches with their syncs)", "ms": round(dt * 1e3, 3),
                    "split_resolve_passes": self.comp.unlz4_resolve_passes()}


def stream_big_leg(data: bytes, reps: int):
    """The drop-in stream path in C++: tools/bin/stream_threads (tests/cpp/stream_threads.cpp, built by
    smallz4_amd/csrc/Makefile) calls smallz4::lz4 through include/smallz4_amd.hpp on `reps` x 100 MB of
    the benchmark text at -9 -- 4 MiB dependent blocks, 64 MiB chunks, callbacks and PCIe both ways in
    the clock -- after a first call of one repetition that allocates the pooled context.  A child
    process: it owns its own context, so its device footprint is its own."""
    exe = os.path.join(ROOT, "tools", "bin", "stream_threads")
    if not os.path.exists(exe):
        return {"skipped": "tools/bin/stream_threads not built"}
    base = "/tmp/sz4_bench_stream_base.bin"
    with open(base, "wb") as f:
        f.write(data[:100_000_000])
    try:
        r = subprocess.run([exe, "big", "9", base, str(reps), "/dev/null", "decode"], capture_output=True, text=True,
                           timeout=400)
    finally:
        os.unlink(base)
    if r.returncode != 0:
        return {"error": f"exit {r.returncode}", "stderr": r.stderr[-500:]}
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    chunks = -(-rec["input_bytes"] // (64 << 20))
    return {"value": rec["MB/s"], "unit": "MB/s (smallz4::lz4 wall clock: callbacks, PCIe both ways, kernels)",
            "input_bytes": rec["input_bytes"], "chunks": chunks, "ratio": round(rec["output_bytes"] / rec["input_bytes"], 5),
            "device_bytes": rec["device_bytes"], "seconds": rec["seconds"],
            "get_bytes_seconds": rec["get_bytes_seconds"], "send_bytes_seconds": rec["send_bytes_seconds"],
            "first_call": {"input_bytes": rec["first_call_bytes"], "seconds": rec["first_call_seconds"]},
            "decode": {"MB/s": rec["decode_MB/s"], "seconds": rec["decode_seconds"], "roundtrip_ok": rec["decode_ok"],
                       "path": "sz4_unlz4_stream (smallz4cat's unlz4_userPtr interface: getByte per byte, 64 KiB "
                               "sendBytes) on the frame above, output compared with the input as it arrives"},
            "path": "tools/bin/stream_threads big: smallz4::lz4 (include/smallz4_amd.hpp) over 4 MiB dependent blocks, "
                    "64 MiB chunks, level -9, " + f"{reps} x 100 MB of the benchmark text (8 bytes patched per repetition)"}


def dictionary_leg(run: Runner, no_verify: bool):
    """Dictionary mode (smallz4::lz4 with a dictionary, sz4_lz4 between host buffers): 8 MB of text with a
    64 KiB dictionary at -9 and -6, diffed against the reference (oracle/_ref), and 8 MB with a 200 KB zero
    run in the middle at -9 (the same-letter shortcut rounds), checked against the reference's own frame
    hash (tests/golden/streams.json: the reference needs ~15 s for it)."""
    import hashlib
    import numpy as np
    from oracle import pyoracle
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import inputs
    dic = synth.enwik8_like(65536, seed=82)
    text = synth.enwik8_like(8_000_000, seed=83)
    with open(os.path.join(ROOT, "tests", "golden", "streams.json")) as f:
        fix = {c["name"]: c for c in json.load(f)["cases"]}["dict_zero_run_8m_l9"]
    cases = [("text_8m_l9", text, dic, 65535, None), ("text_8m_l6", text, dic, 6, None),
             ("zero_run_8m_l9", inputs.make(fix["input"]), inputs.make(fix["dictionary"]), 65535, fix)]
    res = {}
    for name, data, d, chain, want in cases:
        src = np.frombuffer(data, dtype=np.uint8)
        dst = np.empty(run.comp._lib.sz4_lz4_bound(src.size, 0), dtype=np.uint8)
        run.comp.lz4_into(src, dst, chain, d)  # the first call grows the context's buffers to this input
        t0 = time.perf_counter()
        size = run.comp.lz4_into(src, dst, chain, d)
        dt = time.perf_counter() - t0
        out = dst[:size].tobytes()
        rec = {"MB/s": round(len(data) / dt / 1e6, 1), "input_bytes": len(data), "dictionary_bytes": len(d),
               "max_chain": chain, "rounds": run.comp.dict_rounds(), "ratio": round(size / len(data), 5)}
        if want is not None:
            rec.update({"byte_diff": 0 if hashlib.sha256(out).hexdigest() == want["frame_sha256"] else -1,
                        "verified_against": "reference frame SHA-256 (tests/golden/streams.json)"})
        elif not no_verify and pyoracle.ref_available():
            ref = pyoracle.ref_lz4(data, chain, d)
            m = min(len(ref), len(out))
            rec.update({"byte_diff": int(np.count_nonzero(np.frombuffer(ref[:m], np.uint8) != np.frombuffer(out[:m], np.uint8)))
                        + abs(len(ref) - len(out)), "verified_against": "reference"})
        res[name] = rec
    return {"unit": "MB/s (host buffers in and out, PCIe included; second call on the same input timed)", "cases": res,
            "path": "sz4_lz4 with a dictionary: the data-parallel dictionary finder (sz4_dict.hip), then the usual parse"}


LEVELS = (1, 3, 6, 8)


def levels_leg(args, run: Runner, data: bytes, bs: int):
    """configs[1] at the other chain-depth levels the drop-in keeps (smallz4.cpp:232-238: -1..-8 are
    maxChainLength 1..8; -1..-3 greedy, -4..-6 lazy, both with the reference's skip bookkeeping,
    smallz4.h:726-744): GPU MB/s, a sampled byte diff against the reference CLI at that level, and the
    reference's own rate at that level on the host's cores."""
    import smallz4_amd
    torch = run.torch
    res = {}
    for lv in LEVELS:
        chain = smallz4_amd.level_to_chain(lv)
        elapsed, stages, size, out, t_in = run.compress(data, bs, chain, args.level_steps, 1, "none")
        part = out[:size].cpu().numpy().tobytes()
        del out, t_in
        torch.cuda.empty_cache()
        rec = {"level": f"-{lv}", "max_chain": chain, "MB/s": round(len(data) * args.level_steps / elapsed / 1e6, 2),
               "ms_per_step": round(elapsed / args.level_steps * 1e3, 3), "steps": args.level_steps, "warmup": 1,
               "compression_ratio": round((size + 11) / len(data), 5),
               "stages_ms": {k: round(v, 3) for k, v in stages.items()}}
        if not args.no_verify:
            rec.update(verify_sample(part, data, bs, chain, args.verify_threads, args.level_verify_seconds, every=False))
        if args.cpu_seconds > 0:
            rec["cpu_baseline"] = cpu_baseline(data, bs, chain, min(args.cpu_seconds, args.level_cpu_seconds))
        res[f"-{lv}"] = rec
        print(json.dumps({"levels": f"-{lv}", **rec}), file=sys.stderr, flush=True)
        del part
    return {"config": f"configs[1]'s input: {len(data) / 1e6:g} MB as independent {bs}-byte blocks", "levels": res}


def shapes_leg(args, run: Runner, chain: int, enwik8_data: bytes):
    """The other single-GPU-sized configs, each measured, diffed on a bounded sample and round-tripped."""
    torch = run.torch
    res = {}
    for label, wl, bso in SHAPES:
        t0 = time.perf_counter()
        total, lo, hi, bs = rank_range(args, 1, 0, workload=wl, block_size=bso, mb=0)
        if wl == "enwik8" and enwik8_data is not None and len(enwik8_data) == hi - lo:
            data = enwik8_data
        elif wl == "enwik9":
            # configs[3]'s rank-0 slice at N=8: the same 125 MB every rank compresses at any N
            total, lo, hi, bs = rank_range(args, 8, 0, workload=wl, mb=0)
            data = WORKLOADS[wl][4](lo, hi)
        else:
            data = WORKLOADS[wl][4](lo, hi)
        gen_s = time.perf_counter() - t0
        steps = args.shape_steps
        elapsed, stages, size, out, t_in = run.compress(data, bs, chain, steps, 1, "none")
        part = out[:size].cpu().numpy().tobytes()
        rt_ok, rt = run.roundtrip(out, size, "none", t_in, reps=2)
        del out, t_in
        torch.cuda.empty_cache()
        rec = {"config": f"{wl} ({WORKLOADS[wl][0]}): {len(data) / 1e6:g} MB as independent {bs}-byte blocks, "
                         f"level -{args.level}", "baseline_config": WORKLOADS[wl][0], "block_size": bs,
               "input_bytes": len(data), "MB/s": round(len(data) * steps / elapsed / 1e6, 2),
               "ms_per_step": round(elapsed / steps * 1e3, 3), "steps": steps, "warmup": 1,
               "compression_ratio": round((size + 11) / len(data), 5), "roundtrip_ok": rt_ok,
               "stages_ms": {k: round(v, 3) for k, v in stages.items()}, "generate_s": round(gen_s, 1),
               "unlz4": rt}
        if not args.no_verify:
            # configs[2] is diffed in full (every block, `every`), the others on a sample cut at the budget
            full = label == "silesia_4m"
            budget = args.silesia_verify_seconds if full else args.shape_verify_seconds
            rec.update(verify_sample(part, data, bs, chain, args.verify_threads, budget, every=full))
        res[label] = rec
        print(json.dumps({"shape": label, **rec}), file=sys.stderr, flush=True)
        del data, part
    return res


def main():
    args = parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run:
        return dry_run(args, world, rank)

    import torch
    import torch.distributed as dist
    # SZ4_BENCH_SHARE_DEVICE=1: every rank on GPU 0 with gloo collectives -- the sharded path rehearsed on
    # a one-GPU box (tests/test_shards.py); RCCL does not take two ranks on one device
    share = os.environ.get("SZ4_BENCH_SHARE_DEVICE") == "1"
    if share:
        local = 0
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    import smallz4_amd

    chain = smallz4_amd.level_to_chain(args.level)
    total, lo, hi, bs = rank_range(args, world, rank)
    nbytes = hi - lo
    data = WORKLOADS[args.workload][4](lo, hi)
    run = Runner(local)
    # rank 0 writes the smallz4 header, the last rank the end mark, the others bare blocks
    header = "smallz4" if world == 1 else "none"
    barrier = dist.barrier if world > 1 else None
    elapsed, stages, size, out, t_in = run.compress(data, bs, chain, args.steps, args.warmup, header, barrier)
    part = out[:size].cpu().numpy().tobytes()
    blocks = part[7:-4] if header == "smallz4" else part

    # device round trip of this rank's part (outside the timed region)
    rt_ok, dec = True, None
    if not args.no_decode and nbytes:
        rt_ok, dec = run.roundtrip(out, size, header, t_in)
    del out, t_in
    torch.cuda.empty_cache()

    # output-byte diff against the reference: every block at N=1 on enwik8, else a sample bounded in time
    ver = {"byte_diff": -1, "blocks_verified": 0, "verified_against": None}
    if not args.no_verify and nbytes:
        every = world == 1 and args.workload == "enwik8"
        ver = verify_sample(blocks, data, bs, chain, args.verify_threads, 600.0 if every else args.verify_seconds, every)

    # whole-job results over ranks
    res = torch.tensor([elapsed, float(size), float(ver["byte_diff"]), float(ver["blocks_verified"]),
                        0.0 if rt_ok else 1.0], dtype=torch.float64, device="cpu" if share else f"cuda:{local}")
    if world > 1:
        mx = res.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(res, op=dist.ReduceOp.SUM)
        elapsed = float(mx[0])
        frame_bytes = int(res[1]) + 11
        diff = -1 if float(mx[2]) < 0 else int(res[2])
        verified, rt_bad = int(res[3]), int(res[4])
    else:
        frame_bytes, diff, verified, rt_bad = size, ver["byte_diff"], ver["blocks_verified"], 0 if rt_ok else 1

    stream_leg = dict_leg = None
    if world == 1 and not args.no_stream and nbytes:
        stream_leg = stream_big_leg(data, args.stream_reps)
    if world == 1 and not args.no_dict and args.level == 9:
        dict_leg = dictionary_leg(run, args.no_verify)

    levels = None
    if world == 1 and not args.no_levels and args.level == 9 and args.workload == "enwik8" and not args.mb and nbytes:
        levels = levels_leg(args, run, data, bs)

    shapes = None
    if world == 1 and not args.no_shapes and args.level == 9 and args.workload == "enwik8" and not args.mb:
        shapes = shapes_leg(args, run, chain, data)

    if rank == 0:
        wl = WORKLOADS[args.workload]
        value = total * args.steps / elapsed / 1e6
        cfg = {"workload": f"{args.workload} ({wl[0]}): {total / 1e6:g} MB as independent {bs}-byte blocks, "
                           f"level -{args.level} (maxChainLength {chain}), {nbytes / 1e6:g} MB per GPU",
               "baseline_config": wl[0], "block_size": bs, "level": args.level, "input_bytes": total,
               "bytes_per_gpu": nbytes, "parallelism": f"block ranges of one input sharded over {world} GPU(s), "
                                                      "no data-path collective"}
        # dominant kernel k_find_sorted (the sort fused in).  Algorithmic bytes per position: text byte
        # read (1) + the sorted slot arrays written for the later passes (4: u16 position and group
        # start) + the match written (6: u32 length, u16 distance) = 11 B
        find_ms = stages.get("find_sorted", 0.0)
        alg_bytes = 11 * nbytes
        achieved = alg_bytes / (find_ms * 1e-3) / 1e9 if find_ms > 0 else 0.0
        pmc_cfg = {"workload": args.workload, "bytes_per_gpu": nbytes, "block_size": bs, "level": args.level}
        pmc = pmc_traffic(pmc_cfg)
        # The kernel is bound by instruction issue (it checks every candidate of the reference's -9 hash
        # chain), not by HBM: "bound" says so, achieved/peak/frac are its HBM
        # roofline, "issue" its issue roofline from the SQ pass of the PMC profile
        roof = {"kernel": "k_find_sorted (k_sort fused in)", "bound": "issue", "achieved": round(achieved, 3),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                "traffic": pmc[1]["hbm_bytes_per_launch"] if pmc else None,
                "algorithmic_bytes_per_launch": alg_bytes,
                "limiter": "instruction issue and latency (VALU candidate checks, SALU control): achieved/peak is "
                           "the HBM roofline (algorithmic bytes per launch / launch time vs 8 TB/s), the issue "
                           "roofline is under 'issue'",
                "step_compulsory": {"bytes": nbytes + size, "GB/s": round((nbytes + size) / (elapsed / args.steps) / 1e9, 3),
                                    "frac": round((nbytes + size) / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 6),
                                    "note": "input read + frame written per GPU per step over the whole step"}}
        if pmc:
            roof["traffic_source"] = os.path.relpath(pmc[0], ROOT)
            rec_p = pmc[1]
            if rec_p.get("hbm_bytes_per_launch"):
                roof["traffic_over_algorithmic"] = round(rec_p["hbm_bytes_per_launch"] / alg_bytes, 3)
            # issue roofline (MI355X_MICROARCH.md: a wave64 VALU instruction holds a SIMD-32 for 2 cycles
            # -> 0.5 per SIMD-cycle; one scalar unit per CU -> 1 per CU-cycle)
            issue = {"source": os.path.relpath(pmc[0], ROOT), "profiled_avg_duration_us": rec_p.get("avg_duration_us")}
            if rec_p.get("valu_per_simd_cycle") is not None:
                issue.update({"valu_per_simd_cycle": rec_p["valu_per_simd_cycle"], "valu_peak": 0.5,
                              "valu_frac": round(rec_p["valu_per_simd_cycle"] / 0.5, 4)})
                ceil = valu_ceiling()
                if ceil:
                    # the integer VALU rate the chip sustains (tools/valu_ceiling.hip), both at the clocks
                    # measured while each ran (the kernel's from its SQ pass: GRBM_GUI_ACTIVE over the time)
                    mine = rec_p.get("valu_per_simd_cycle_at_clock", rec_p["valu_per_simd_cycle"])
                    issue.update({"valu_per_simd_cycle_at_clock": mine,
                                  "clock_ghz_measured": rec_p.get("clock_ghz_measured"),
                                  "valu_ceiling_measured": ceil["vgpr"], "valu_ceiling_clock_ghz": ceil["clock_ghz"],
                                  "valu_ceiling_sgpr_operands": ceil.get("sgpr"),
                                  "valu_frac_of_measured": round(mine / ceil["vgpr"], 4),
                                  "valu_ceiling_source": ceil["source"]})
            if rec_p.get("salu_per_cu_cycle") is not None:
                issue.update({"salu_per_cu_cycle": rec_p["salu_per_cu_cycle"], "salu_peak": 1.0,
                              "salu_frac": round(rec_p["salu_per_cu_cycle"], 4)})
            roof["issue"] = issue
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
            "data": wl[1],
            "config": cfg,
            "value_per_gpu": round(value / world, 2),
            "byte_diff": diff,
            "blocks_verified": verified,
            "verified_against": ver.get("verified_against"),
            "verify": {k: v for k, v in ver.items() if k.startswith("verify") or k == "blocks_total"},
            "roundtrip_ok": rt_bad == 0,
            "compression_ratio": round(frame_bytes / total, 5) if total else None,
            "stages_ms": {k: round(v, 3) for k, v in stages.items()},
            "roofline": roof,
        }
        if dec is not None:
            rec["unlz4"] = dec
        if stream_leg is not None:
            rec["stream"] = stream_leg
        if dict_leg is not None:
            rec["dictionary"] = dict_leg
        if levels is not None:
            rec["levels"] = levels
        if shapes is not None:
            rec["shapes"] = shapes
        # the reference on this host's cores, rank 0, after the timed region (at every N)
        rec["cpu_baseline"] = cpu_baseline(data, bs, chain, args.cpu_seconds)
        print(json.dumps(rec), flush=True)
        print(summary_line(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
