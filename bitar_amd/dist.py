"""Multi-GPU sharding of one job's segments and the global frame index.

Every segment is an independent op (reference src/memory.cc:110), so ranks never exchange
payload.  A job of `nseg` segments is cut into batches of `batch` consecutive segments that
are dealt round-robin to the ranks -- the reference demo's even split + round-robin device
choice (apps/demo_app.cc:249-256 `Advance`, 579-596).  Inside a rank, its segments are laid
out contiguously in ascending global order and split evenly into one part per queue-pair
stream (the demo's split of the input into lcores-1 parts, each handed to one queue pair).
Each rank compresses its parts on its own GPU; the one collective is an all-gather of the
per-segment compressed sizes (uint32), from which every rank builds the same global frame
index: the byte offset of every segment's frame in the job's packed output, in global
segment order.  Decompression needs no collective.

The collective runs over whatever process group torch.distributed was initialised with:
RCCL ("nccl") between GPUs, gloo in the CPU tests.  Nothing here touches a GPU by itself.
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


@dataclass(frozen=True)
class Run:
    """One batch of a rank: global segments [gseg, gseg + count) stored at local segment
    index `lseg`; bytes [goff, goff + nbytes) of the job at local byte `loff`."""
    gseg: int
    lseg: int
    count: int
    goff: int
    loff: int
    nbytes: int


@dataclass(frozen=True)
class Part:
    """The share of one queue-pair stream: local segments [lseg, lseg + count), local bytes
    [loff, loff + nbytes)."""
    stream: int
    lseg: int
    count: int
    loff: int
    nbytes: int


class Layout:
    """Where a rank's share of a job lives in its HBM buffers (pure bookkeeping).

    job_bytes are cut into `seg`-byte segments (the last may be short); batches of `batch`
    segments go round-robin to the ranks (assign); the rank stores its segments contiguously
    (input at local byte lseg*seg, slot at lseg*stride, size/produced at lseg) and splits
    them into `nstreams` near-equal parts of whole segments.
    """

    def __init__(self, job_bytes: int, seg: int, world: int = 1, rank: int = 0,
                 nstreams: int = 1, batch: int = 256):
        if seg < 1 or job_bytes < 0 or nstreams < 1:
            raise ValueError("bad job parameters")
        self.job_bytes, self.seg, self.world, self.rank = job_bytes, seg, world, rank
        self.batch, self.nstreams = batch, nstreams
        self.nseg = (job_bytes + seg - 1) // seg
        self.shard = assign(self.nseg, world, rank, batch)
        runs = []
        lseg = 0
        loff = 0
        nbatch = (self.nseg + batch - 1) // batch
        for b in range(rank, nbatch, world):
            g0 = b * batch
            cnt = min(batch, self.nseg - g0)
            goff = g0 * seg
            nb = min(cnt * seg, job_bytes - goff)
            runs.append(Run(g0, lseg, cnt, goff, loff, nb))
            lseg += cnt
            loff += nb
        self.runs = runs
        self.local_nseg = lseg
        self.local_bytes = loff
        parts = []
        per, extra = divmod(lseg, nstreams)
        s0 = 0
        for k in range(nstreams):
            cnt = per + (1 if k < extra else 0)
            if cnt == 0:
                continue
            b0 = s0 * seg
            b1 = min((s0 + cnt) * seg, loff)
            parts.append(Part(k, s0, cnt, b0, b1 - b0))
            s0 += cnt
        self.parts = parts


class SizeGather:
    """The job's one collective: all-gather every rank's per-segment compressed sizes and
    put them in global segment order (the gather order is precomputed once, so each call is
    one all-gather + one index_select on the sizes' device)."""

    def __init__(self, nseg: int, world: int, batch: int = 256, device=None):
        self.nseg, self.world, self.batch = nseg, world, batch
        shards = [assign(nseg, world, r, batch).segments for r in range(world)]
        self.cap = max((s.numel() for s in shards), default=0)
        src = torch.empty(nseg, dtype=torch.int64)
        for r, s in enumerate(shards):
            src[s] = r * self.cap + torch.arange(s.numel(), dtype=torch.int64)
        self.src = src.to(device) if device is not None else src
        self.device = device

    def __call__(self, local_sizes: torch.Tensor, group=None) -> torch.Tensor:
        """local_sizes: this rank's sizes in local order (int32 holding uint32 values).
        Returns int64 [nseg] in global order."""
        import torch.distributed as dist
        dev = local_sizes.device
        padded = torch.zeros(self.cap, dtype=torch.int32, device=dev)
        padded[:local_sizes.numel()] = local_sizes.to(torch.int32)
        gathered = torch.empty(self.world * self.cap, dtype=torch.int32, device=dev)
        # the collective runs whenever a process group is up -- at world size 1 too (a
        # one-rank RCCL group under torch.distributed.run), so that path is exercised on one GPU
        coll = self.world > 1 or (dist.is_available() and dist.is_initialized())
        if coll and dev.type == "cuda" and dist.get_backend(group) != "nccl":
            # gloo gathers host tensors (the CPU tests, the one-GPU rehearsal)
            g = torch.empty(self.world * self.cap, dtype=torch.int32)
            dist.all_gather_into_tensor(g, padded.cpu(), group=group)
            gathered.copy_(g)
        elif coll:
            dist.all_gather_into_tensor(gathered, padded, group=group)
        else:
            gathered = padded  # (one rank, no group: the sizes are the whole gather)
        src = self.src if self.src.device == dev else self.src.to(dev)
        return gathered.index_select(0, src).to(torch.int64) & 0xFFFFFFFF


def gather_sizes(local_sizes: torch.Tensor, nseg: int, world: int, batch: int = 256,
                 group=None) -> torch.Tensor:
    """All-gather every rank's per-segment compressed sizes and return them in global
    segment order (int64 [nseg]).  `local_sizes` holds this rank's sizes in the order of
    assign(...).segments (uint32 values in an int32 tensor, as the kernels write them)."""
    return SizeGather(nseg, world, batch)(local_sizes, group=group)


def frame_index(sizes: torch.Tensor) -> torch.Tensor:
    """Exclusive prefix sum of the global per-segment sizes: offsets[i] = start of segment
    i's frame in the packed job output; offsets[nseg] = total compressed bytes."""
    off = torch.zeros(sizes.numel() + 1, dtype=torch.int64, device=sizes.device)
    torch.cumsum(sizes.to(torch.int64), 0, out=off[1:])
    return off
