"""Multi-GPU sharding of one job's segments and the global frame index.

Every segment is an independent op (reference src/memory.cc:110), so ranks never exchange
payload.  A job of `nseg` segments is cut into batches of `batch` consecutive segments that
are dealt round-robin to the ranks -- the reference demo's even split + round-robin device
choice (apps/demo_app.cc:249-256, 579-596).  Each rank compresses its batches on its own GPU;
the one collective is an all-gather of the per-segment compressed sizes (uint32), from which
every rank builds the same global frame index: the byte offset of every segment's frame in
the job's packed output, in global segment order.  Decompression needs no collective.

The collective runs over whatever process group torch.distributed was initialised with:
RCCL ("nccl") between GPUs, gloo in the CPU tests.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch


@dataclass(frozen=True)
class Shard:
    """The segments of one rank: `segments` are global segment ids, ascending."""
    rank: int
    segments: torch.Tensor  # int64 [k]


def assign(nseg: int, world: int, rank: int, batch: int = 256) -> Shard:
    """Global segment ids owned by `rank`: batches b = rank, rank + world, ...; each batch
    is segments [b*batch, min((b+1)*batch, nseg))."""
    if world < 1 or not 0 <= rank < world or batch < 1 or nseg < 0:
        raise ValueError("bad sharding parameters")
    nbatch = (nseg + batch - 1) // batch
    ids = [torch.arange(b * batch, min((b + 1) * batch, nseg), dtype=torch.int64)
           for b in range(rank, nbatch, world)]
    segs = torch.cat(ids) if ids else torch.empty(0, dtype=torch.int64)
    return Shard(rank, segs)


def max_shard_len(nseg: int, world: int, batch: int = 256) -> int:
    return max(assign(nseg, world, r, batch).segments.numel() for r in range(world))


def gather_sizes(local_sizes: torch.Tensor, nseg: int, world: int, batch: int = 256,
                 group=None) -> torch.Tensor:
    """All-gather every rank's per-segment compressed sizes and return them in global
    segment order (int64 [nseg]).  `local_sizes` holds this rank's sizes in the order of
    assign(...).segments (uint32 values in an int32 tensor, as the kernels write them)."""
    import torch.distributed as dist
    cap = max_shard_len(nseg, world, batch)
    padded = torch.zeros(cap, dtype=torch.int32, device=local_sizes.device)
    padded[:local_sizes.numel()] = local_sizes.to(torch.int32)
    gathered = torch.empty(world * cap, dtype=torch.int32, device=local_sizes.device)
    if world > 1:
        dist.all_gather_into_tensor(gathered, padded, group=group)
    else:
        gathered.copy_(padded)
    out = torch.empty(nseg, dtype=torch.int64, device=local_sizes.device)
    g = gathered.view(world, cap).to(torch.int64) & 0xFFFFFFFF
    for r in range(world):
        segs = assign(nseg, world, r, batch).segments.to(local_sizes.device)
        out[segs] = g[r, :segs.numel()]
    return out


def frame_index(sizes: torch.Tensor) -> torch.Tensor:
    """Exclusive prefix sum of the global per-segment sizes: offsets[i] = start of segment
    i's frame in the packed job output; offsets[nseg] = total compressed bytes."""
    off = torch.zeros(sizes.numel() + 1, dtype=torch.int64, device=sizes.device)
    torch.cumsum(sizes.to(torch.int64), 0, out=off[1:])
    return off
