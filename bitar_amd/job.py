"""One rank's share of a sharded compress / decompress job on its GPU (SURVEY.md §8e,
BASELINE configs[2] and [3]).

The job's layout comes from bitar_amd.dist.Layout: round-robin batches of segments per rank,
the rank's segments contiguous in HBM, split into one part per queue-pair stream.  Each
part is ONE kernel launch on its stream (the reference's per-queue-pair Compress /
Decompress calls, device.cc:156-318, launched asynchronously on their lcores by
CompressAsync / DecompressAsync, util.h:216-236); the streams run concurrently.  After the
compress launches, the per-segment sizes are all-gathered (RCCL) and every rank builds the
global frame index; decompression of each part follows its compress on the same stream, so
it overlaps the all-gather.
"""
from __future__ import annotations

import torch

import bitar_amd
from bitar_amd import dist as bd


class ShardedJob:
    def __init__(self, eng: "bitar_amd.Engine", codec: int, job_bytes: int, seg: int,
                 world: int = 1, rank: int = 0, nstreams: int = 1, batch: int = 256,
                 group=None):
        if (batch * seg) % 64:
            raise ValueError("batch * seg must be a multiple of 64 (generator lines)")
        self.eng, self.codec, self.group = eng, codec, group
        self.layout = L = bd.Layout(job_bytes, seg, world, rank, nstreams, batch)
        self.seg = seg
        self.stride = bitar_amd.slot_size(codec, seg)
        self.world = world
        dev = f"cuda:{eng.device}"
        self.data = eng.empty(max(L.local_bytes, 1))
        self.slab = eng.empty(max(L.local_nseg * self.stride, 1))
        self.sizes = eng.empty(max(L.local_nseg, 1), dtype=torch.int32)
        self.out = eng.empty(max(L.local_nseg * seg, 1))
        self.produced = eng.empty(max(L.local_nseg, 1), dtype=torch.int32)
        self.gather = bd.SizeGather(L.nseg, world, batch, device=dev)
        self.index = None
        # one stream per part: torch's current stream when there is a single part (so
        # torch events / collectives need no cross-stream wait), else queue-pair streams
        if nstreams == 1:
            self.streams = [None]
        else:
            self.streams = [eng.queue_pair_stream(k) for k in range(nstreams)]
        self.tstreams = [torch.cuda.current_stream(eng.device) if s is None else
                         torch.cuda.ExternalStream(s, device=dev) for s in self.streams]

    # -- input -----------------------------------------------------------------------------
    def generate(self, kind: int, seed: int):
        """The rank's batches of the deterministic job stream (kind, seed), in HBM."""
        for r in self.layout.runs:
            self.eng.fill(kind, seed, self.data[r.loff:], n=r.nbytes, offset=r.goff)

    # -- the step ----------------------------------------------------------------------------
    def compress(self, events=None):
        # a part's stream must not overwrite sizes the previous step's gather still reads
        cur = torch.cuda.current_stream(self.eng.device)
        for ts in self.tstreams:
            if ts != cur:
                ts.wait_stream(cur)
        for p in self.layout.parts:
            s = self.streams[p.stream]
            ev = events.get(p.stream) if events is not None else None
            if ev is not None:
                ev[0].record(self.tstreams[p.stream])
            self.eng.compress_into(self.codec, self.data[p.loff:], self.seg,
                                   self.slab[p.lseg * self.stride:], self.stride,
                                   self.sizes[p.lseg:], n=p.nbytes, stream=s)
            if ev is not None:
                ev[1].record(self.tstreams[p.stream])

    def gather_index(self):
        """RCCL all-gather of the sizes + global frame index (after every part's compress)."""
        cur = torch.cuda.current_stream(self.eng.device)
        for p in self.layout.parts:
            ts = self.tstreams[p.stream]
            if ts != cur:
                cur.wait_stream(ts)
        sizes = self.gather(self.sizes[:self.layout.local_nseg], group=self.group)
        self.index = bd.frame_index(sizes)
        return self.index

    def decompress(self, events=None):
        for p in self.layout.parts:
            s = self.streams[p.stream]
            ev = events.get(p.stream) if events is not None else None
            if ev is not None:
                ev[0].record(self.tstreams[p.stream])
            self.eng.decompress_slab_into(self.codec, self.slab[p.lseg * self.stride:],
                                          self.stride, self.sizes[p.lseg:], p.count, self.seg,
                                          self.out[p.lseg * self.seg:],
                                          self.produced[p.lseg:], capacity=p.count * self.seg,
                                          stream=s)
            if ev is not None:
                ev[1].record(self.tstreams[p.stream])

    def step(self):
        self.compress()
        self.gather_index()
        self.decompress()

    # -- checks ------------------------------------------------------------------------------
    def sync(self):
        """Wait for every stream; raises BitarError if any op of this job failed."""
        for s in self.streams:
            self.eng.sync(s)

    def verify(self) -> bool:
        """Byte equality of the round trip (demo_app.cc:534-543, 671-686) and the frame
        index spans this rank's sizes."""
        torch.cuda.synchronize(self.eng.device)
        L = self.layout
        n = L.local_bytes
        ok = bool(torch.equal(self.out[:n], self.data[:n]))
        ok = ok and int(self.produced[:L.local_nseg].to(torch.int64).sum().item()) == n
        return ok

    def local_compressed_bytes(self) -> int:
        return int(self.sizes[:self.layout.local_nseg].to(torch.int64).sum().item())

    def free(self):
        del self.data, self.slab, self.out, self.sizes, self.produced
        torch.cuda.empty_cache()
