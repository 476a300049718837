"""Sharding of independent blocks across ranks (one process per GPU).

Blocks are independent, so a job partitions into contiguous block ranges with no
data-path collective: each rank compresses its range with the header suppressed
("none"), and the frame is the concatenation of the parts in rank order, with the
smallz4 header in front and the end mark behind -- byte-identical to compressing
the whole input on one GPU.  Gathering the parts is optional (gather_frame);
nothing in the compression itself communicates.
"""
from __future__ import annotations

HEADER = bytes([0x04, 0x22, 0x4D, 0x18, 0x40, 0x70, 0xDF])
END_MARK = b"\0\0\0\0"


def shard_range(n: int, block_size: int, rank: int, world: int) -> tuple[int, int]:
    """Byte range [lo, hi) of the blocks rank `rank` of `world` compresses (contiguous, balanced)."""
    if not (0 <= rank < world) or block_size <= 0:
        raise ValueError("bad rank/world/block_size")
    nblocks = (n + block_size - 1) // block_size
    b0 = nblocks * rank // world
    b1 = nblocks * (rank + 1) // world
    return min(n, b0 * block_size), min(n, b1 * block_size)


def frame_part(body: bytes, rank: int, world: int) -> bytes:
    """Wrap a rank's bare blocks so that concatenating all parts gives the full frame."""
    return (HEADER if rank == 0 else b"") + body + (END_MARK if rank == world - 1 else b"")


def gather_frame(part: bytes, group=None) -> bytes:
    """Concatenate every rank's part (torch.distributed all_gather_object)."""
    import torch.distributed as dist
    parts = [None] * dist.get_world_size(group)
    dist.all_gather_object(parts, part, group=group)
    return b"".join(parts)
