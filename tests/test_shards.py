"""The sharded configurations on one MI355X: BASELINE configs[3] (enwik9-shaped, 64 KiB blocks) and
configs[4] (zeros/urandom, 256 KiB blocks) as the 8-GPU run splits them, one rank's slice at full
size.  Blocks are independent, so a rank's part is bare blocks and the rank-ordered parts concatenate
to the single-GPU frame.  Full-size slices are checked through size-independent properties (device
round trip, the size-word walk) plus the oracle on a fixed sample of blocks.  Run with -m gpu."""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import pyoracle
from smallz4_amd import shard, synth

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _device_roundtrip(compressor, part: bytes, data: bytes):
    import torch
    frame = shard.HEADER + part + shard.END_MARK
    f = torch.frombuffer(bytearray(frame), dtype=torch.uint8).cuda()
    want = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    out = torch.empty(len(data), dtype=torch.uint8, device="cuda")
    n = compressor.unlz4_device(f.data_ptr(), len(frame), out.data_ptr(), len(data))
    torch.cuda.synchronize()
    return n == len(data) and bool(torch.equal(out, want))


def _spans(part: bytes):
    spans, pos = [], 0
    while pos + 4 <= len(part):
        word = int.from_bytes(part[pos:pos + 4], "little")
        spans.append((pos, 4 + (word & 0x7FFFFFFF)))
        pos += 4 + (word & 0x7FFFFFFF)
    assert pos == len(part)
    return spans


def _zu_fixtures(prefix):
    """{block index: (SHA-256, length)} of the reference's bytes for the sampled configs[4] blocks
    (tests/golden/make_blocks_golden.py, one single-block case per sampled block)."""
    with open(os.path.join(ROOT, "tests", "golden", "blocks.json")) as f:
        cases = json.load(f)["cases"]
    return {int(c["name"][len(prefix):]): (c["block_sha256"][0], c["block_len"][0])
            for c in cases if c["name"].startswith(prefix)}


def test_two_contexts_shards_concatenate_to_single_frame(compressor):
    """Two ranks' work on one GPU: two contexts, one per shard of ONE input, header 'none'."""
    import smallz4_amd
    data = synth.enwik9_like_range(0, 9_000_000)
    bs = 65536
    other = smallz4_amd.Compressor(device=0)
    parts = []
    for r, comp in enumerate((compressor, other)):
        lo, hi = shard.shard_range(len(data), bs, r, 2)
        parts.append(shard.frame_part(comp.compress_blocks(data[lo:hi], bs, 65535, header="none"), r, 2))
    assert b"".join(parts) == compressor.compress_blocks(data, bs, 65535)
    other.close()


@pytest.mark.parametrize("workload,world,bs", [("enwik9", 8, 65536), ("zeros_urandom", 8, 262144)])
def test_rank0_slice_full_size(compressor, workload, world, bs):
    """Rank 0's slice of the 8-GPU configuration at full size: 125 MB of configs[3], 1.25 GiB of
    configs[4]."""
    if workload == "enwik9":
        total = 125_000_000 * world
        lo, hi = shard.shard_range(total, bs, 0, world)
        data = synth.enwik9_like_range(lo, hi, seed=9, workers=8)
    else:
        total = (10 << 30)
        lo, hi = shard.shard_range(total, bs, 0, world)
        data = synth.zeros_urandom_range(lo, hi, seed=10)
    # a rank's process runs only its batch calls: what earlier tests left in the shared session context
    # (decoder, stream and dictionary buffers) is released first
    before = compressor.device_bytes()
    compressor.trim()
    part = compressor.compress_blocks(data, bs, 65535, header="none")
    footprint = compressor.device_bytes()  # before the decoder's own scratch joins it
    spans = _spans(part)
    assert len(spans) == (len(data) + bs - 1) // bs
    assert _device_roundtrip(compressor, part, data)
    # a fixed sample of blocks, the first and the last included: enwik9-shaped ones against the oracle,
    # zeros/urandom ones against the reference's own bytes (tests/golden/blocks.json, zu_slice_*: the
    # reference needs ~13 s per such block -- its chain walk is quadratic in a run)
    if workload == "enwik9":
        idx = sorted(set(list(range(0, len(spans), max(1, len(spans) // 24))) + [len(spans) - 1]))
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=8) as ex:
            want = list(ex.map(lambda i: pyoracle.oz_block(data[i * bs:(i + 1) * bs], 65535), idx))
        for i, w in zip(idx, want):
            o, n = spans[i]
            assert part[o:o + n] == w, i
    else:
        fix = _zu_fixtures("zu_slice_")
        assert sorted(fix) == [0, 1706, 3412, 5118, len(spans) - 1]
        for i, (sha, n) in fix.items():
            o, got = spans[i]
            assert got == n and hashlib.sha256(part[o:o + n]).hexdigest() == sha, i
    # HBM footprint of the context for this slice (grow-only scratch)
    print(f"{workload} rank-0 slice {len(data)} B: context holds {footprint / 2**30:.2f} GiB "
          f"({footprint / len(data):.1f} B per input byte; {before / 2**30:.2f} GiB before)")
    # bounded: sz4_compress_blocks_device runs equal pieces of at most 448 MiB (36-49 B of scratch per piece
    # byte), whatever the slice's length
    assert footprint < 24 << 30


def _batch_4gib(compressor, torch):
    """4 GiB of configs[4]'s shape (zeros/urandom runs, 256 KiB blocks) in ONE sz4_compress_blocks_device
    call: the context's scratch stays under 24 GiB (under the bound the call runs pieces of about 1/64 of it,
    384 MiB), the frame decodes
    back on the device, every size word walks, and sampled blocks equal the reference's.  Run by
    tests/test_memory.py on the shared session context under a 24 GiB device bound."""
    bs = 262144
    lo = 3 << 30
    data = synth.zeros_urandom_range(lo, lo + (4 << 30), seed=10)
    t = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    cap = compressor._lib.sz4_bound(len(data), bs)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    size = compressor.compress_blocks_device(t.data_ptr(), len(data), out.data_ptr(), cap, bs, 65535, "none", stream)
    footprint = compressor.device_bytes()
    print(f"4 GiB in one call: context holds {footprint / 2**30:.2f} GiB")
    assert footprint < 24 << 30
    # round trip on the device
    fr = torch.empty(size + 11, dtype=torch.uint8, device="cuda")
    fr[:7] = torch.tensor(list(shard.HEADER), dtype=torch.uint8)
    fr[7:7 + size] = out[:size]
    fr[7 + size:] = 0
    del out
    dec = torch.empty(len(data), dtype=torch.uint8, device="cuda")
    n = compressor.unlz4_device(fr.data_ptr(), fr.numel(), dec.data_ptr(), len(data), stream=stream)
    torch.cuda.synchronize()
    assert n == len(data) and bool(torch.equal(dec, t))
    part = fr[7:7 + size].cpu().numpy().tobytes()
    del fr, dec, t
    spans = _spans(part)
    assert len(spans) == len(data) // bs
    sizes = compressor.last_block_sizes(len(spans))
    assert sizes == [n for _, n in spans]
    # sampled blocks against the reference's own bytes (tests/golden/blocks.json, zu_4g_*)
    fix = _zu_fixtures("zu_4g_")
    assert sorted(fix) == [1, len(spans) // 2 + 3, len(spans) - 1]
    for i, (sha, n) in fix.items():
        o, got = spans[i]
        assert got == n and hashlib.sha256(part[o:o + n]).hexdigest() == sha, i


def test_batch_pieces_equal_one_run(compressor):
    """The internal pieces are invisible: a call forced into 1 MiB pieces writes the same frame (and
    block sizes) as one run over the whole input."""
    data = synth.enwik8_like(5 << 20, seed=91) + bytes(300000) + synth.zeros_urandom_range(0, 3 << 20)
    whole = compressor.compress_blocks(data, 65536, 65535)
    compressor.set_batch_chunk(1 << 20)
    try:
        pieces = compressor.compress_blocks(data, 65536, 65535)
        sizes = compressor.last_block_sizes(200)
    finally:
        compressor.set_batch_chunk(0)
    assert pieces == whole
    assert sum(sizes) == len(whole) - 11 and len(sizes) == (len(data) + 65535) // 65536


@pytest.mark.parametrize("workload,mb,sample", [("enwik9", 8, 16), ("zeros_urandom", 4, 2)])
def test_bench_two_ranks_shard_one_input(workload, mb, sample):
    """`bench.py --gpus 2` end to end on the one-GPU box: two processes (a torch.distributed.run child
    started by bench.py itself), each compressing its block range of ONE input through the HIP
    library; both ranks on GPU 0 with gloo collectives (SZ4_BENCH_SHARE_DEVICE=1; the 8-GPU run uses
    RCCL, one device per rank).  The line must report 2 ranks, the whole input, a zero byte diff on
    every rank's sample and both device round trips."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, SZ4_BENCH_SHARE_DEVICE="1")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--workload", workload,
                        "--mb", str(mb), "--steps", "2", "--warmup", "1", "--verify-seconds", "15",
                        "--cpu-seconds", "1", "--no-stream"], capture_output=True, text=True, timeout=400, cwd=root,
                       env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["n_gpus"] == 2 and rec["config"]["input_bytes"] == 2 * mb * 1_000_000, rec
    assert rec["byte_diff"] == 0 and rec["blocks_verified"] >= sample and rec["roundtrip_ok"], rec
    # the N>1 line carries the CPU baseline (rank 0) and its per-GPU rate, like the N=1 line
    assert rec["cpu_baseline"]["value"] > 0 and rec["value_per_gpu"] * 2 == pytest.approx(rec["value"], rel=1e-3)
    assert rec["verify"]["verify_budget_s"] == 15
