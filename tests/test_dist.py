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
