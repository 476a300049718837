"""Multi-process path on CPU (gloo, world size 2): block ranges partition the input, the
rank-ordered parts concatenate to the single-process frame, and the timing reduction takes
the max over ranks.  The per-block compressor here is the oracle (CPU stand-in for the GPU
kernel, which the -m gpu tests check separately)."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from smallz4_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, bs, q):
    import sys
    import torch
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from oracle import pyoracle
    from smallz4_amd import shard, synth
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    data = synth.enwik8_like(n, seed=77)
    lo, hi = shard.shard_range(n, bs, rank, world)
    body = b"".join(pyoracle.oz_block(data[o:min(o + bs, hi)], 65535) for o in range(lo, hi, bs))
    frame = shard.gather_frame(shard.frame_part(body, rank, world))
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        single = shard.HEADER + b"".join(pyoracle.oz_block(data[o:o + bs], 65535)
                                         for o in range(0, n, bs)) + shard.END_MARK
        q.put((frame == single, float(t.item()), len(frame)))
    dist.destroy_process_group()


@pytest.mark.parametrize("n,bs", [(600000, 65536), (65536 * 3 + 17, 65536), (1000, 65536)])
def test_two_rank_shards_concatenate_to_single_frame(n, bs):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, bs, q)) for r in range(2)]
    for p in procs:
        p.start()
    same, tmax, size = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert same
    assert tmax == 2.0


def test_shard_range_partitions():
    for n in (0, 1, 65535, 65536, 65537, 10 ** 8):
        for world in (1, 2, 3, 8):
            ranges = [shard.shard_range(n, 65536, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            for (a, b), (c, d) in zip(ranges, ranges[1:]):
                assert b == c and a <= b
                assert a % 65536 == 0


def test_bench_gpus2_dry_run_starts_two_ranks():
    """`bench.py --gpus 2` outside torch.distributed starts two ranks itself (torch.distributed.run
    child); in the HIP-free dry run each rank compresses its block range of ONE input (the oracle as
    the block compressor) and the rank-ordered parts equal the single-process frame."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for workload, mb in (("enwik9", 0.3), ("zeros_urandom", 0.6)):
        r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run",
                            "--workload", workload, "--mb", str(mb)],
                           capture_output=True, text=True, timeout=600, cwd=root)
        assert r.returncode == 0, r.stderr[-2000:]
        line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
        rec = json.loads(line)
        assert rec["n_gpus"] == 2 and rec["dry_run"] and rec["parts_equal_single"], rec
        assert rec["input_bytes"] == 2 * int(mb * 1e6)
        # the N > 1 line carries what north_star asks at every N: the workload (the same one the N=1
        # shapes leg runs for configs[3]), the host-CPU baseline with its core count, a bounded verify leg
        assert rec["workload"] == workload
        assert rec["cpu_baseline"]["value"] > 0 and rec["cpu_baseline"]["cores"] >= 1, rec["cpu_baseline"]
        assert 0 < rec["verify_budget_s"] <= 60


def test_range_generators_are_slices_of_one_input():
    from smallz4_amd import synth
    import numpy as np
    a = synth.zeros_urandom_range(0, 40 << 20)
    assert synth.zeros_urandom_range(123457, 777777) == a[123457:777777]
    cell = synth.ZU_CELL
    assert synth.zeros_urandom_range(cell - 5000, cell + 5000) == a[cell - 5000:cell + 5000]
    # configs[4]'s layout: half the bytes zero, zero runs starting at every phase of the 256 KiB grid
    x = np.frombuffer(a, dtype=np.uint8)
    assert 0.45 < (x == 0).mean() < 0.56
    z = np.zeros(len(x) // 4096, dtype=bool)
    z[:] = (x[:len(z) * 4096].reshape(-1, 4096) == 0).all(axis=1)  # 4 KiB pages of zeros
    starts = np.flatnonzero(z[1:] & ~z[:-1]) + 1
    phases = set(((starts * 4096) % 262144) // 32768)
    assert len(starts) > 50 and phases == set(range(8))
    seg = synth.ENWIK9_SEGMENT
    x = synth.enwik9_like_range(seg - 1000, seg + 1000)
    assert x == synth.enwik9_like_range(seg - 1000, seg) + synth.enwik9_like_range(seg, seg + 1000)
