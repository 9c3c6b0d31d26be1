"""Multi-rank sharding + size all-gather + global frame index (bitar_amd/dist.py), on CPU
with the gloo backend at world_size 2 and 3.

Each rank compresses only the segments it was dealt (with the oracle, standing in for the
rank's GPU), the ranks all-gather the per-segment sizes, and every rank must then hold the
same global frame index as a single-process compression of the whole job; the frames
packed in index order must decode back to the input.
"""
import os
import socket

import numpy as np
import pytest

import oracle_lib as O

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from bitar_amd import dist as bd  # noqa: E402

SEG = 4096
N = 37 * SEG + 1234  # 38 segments, ragged tail
BATCH = 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _job():
    return O.fill(O.KIND_MIXED, 5, N)


def _rank_main(rank, world, port, codec, q):
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        data = _job()
        nseg = (N + SEG - 1) // SEG
        shard = bd.assign(nseg, world, rank, BATCH)
        local, frames = [], {}
        for g in shard.segments.tolist():
            src = data[g * SEG:min((g + 1) * SEG, N)].tobytes()
            r, c = O.lz4_compress(src) if codec == O.CODEC_LZ4 else O.deflate_fixed(src)
            assert r == 0
            local.append(len(c))
            frames[g] = c
        sizes = bd.gather_sizes(torch.tensor(local, dtype=torch.int32), nseg, world, BATCH)
        index = bd.frame_index(sizes)
        # every rank places its own frames into the packed job image; a SUM all-reduce
        # assembles it (test plumbing only: the product never moves payload across ranks)
        total = int(index[-1])
        image = torch.zeros(total, dtype=torch.uint8)
        for g, c in frames.items():
            image[int(index[g]):int(index[g]) + len(c)] = torch.frombuffer(bytearray(c), dtype=torch.uint8)
        image32 = image.to(torch.int32)
        dist.all_reduce(image32)
        q.put((rank, sizes.tolist(), index.tolist(), bytes(image32.to(torch.uint8).numpy())))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as ex:  # pragma: no cover - reported to the parent
        q.put((rank, "error", repr(ex), None))


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("codec", [O.CODEC_LZ4, O.CODEC_DEFLATE])
def test_sharded_job_matches_single_process(world, codec):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, codec, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1] != "error", r
    # single-process reference: the whole job, segment by segment
    data = _job()
    nseg = (N + SEG - 1) // SEG
    ref_sizes, blobs = [], []
    for g in range(nseg):
        src = data[g * SEG:min((g + 1) * SEG, N)].tobytes()
        r, c = O.lz4_compress(src) if codec == O.CODEC_LZ4 else O.deflate_fixed(src)
        ref_sizes.append(len(c))
        blobs.append(c)
    ref_index = [0]
    for s in ref_sizes:
        ref_index.append(ref_index[-1] + s)
    for rank, sizes, index, image in res:
        assert sizes == ref_sizes, rank
        assert index == ref_index, rank
        assert image == b"".join(blobs), rank
    # the packed image decodes back to the job
    image = res[0][3]
    out = bytearray()
    for g in range(nseg):
        c = image[ref_index[g]:ref_index[g + 1]]
        if codec == O.CODEC_LZ4:
            r, plain = O.lz4_decompress(c, SEG)
        else:
            r, plain = O.inflate(c, SEG)
        assert r == 0
        out += plain
    assert bytes(out) == data.tobytes()


def test_assign_covers_every_segment_once():
    for nseg in (0, 1, 7, 256, 1000, 131072):
        for world in (1, 2, 3, 8):
            seen = torch.cat([bd.assign(nseg, world, r, 256).segments for r in range(world)])
            assert sorted(seen.tolist()) == list(range(nseg))
    # round-robin batches: rank r gets batches r, r+world, ...
    s = bd.assign(1000, 4, 1, 256).segments.tolist()
    assert s == list(range(256, 512))
    with pytest.raises(ValueError):
        bd.assign(10, 2, 2)


def test_frame_index_single_rank():
    sizes = torch.tensor([5, 0, 7, 0xFFFF], dtype=torch.int64)
    assert bd.frame_index(sizes).tolist() == [0, 5, 5, 12, 12 + 0xFFFF]


# ---- world size 8 rehearsal (the 8-GPU node's rank count) ----------------------------------
# BASELINE configs[3]: an 8 GiB record batch in 64 KiB chunks (131072 segments, 4 queue-pair
# streams per rank); configs[4]: 8 GiB of Zstd column buffers in 64 KiB segments over 2
# streams.  Each rank builds its Layout, makes up deterministic per-segment sizes for the
# segments it owns (a hash of the global id: no compression here, the bookkeeping is under
# test), all-gathers them with SizeGather over gloo and builds the frame index; every rank
# must hold the same global sizes and index as a single-process computation, and the ranks'
# runs must cover every segment and byte of the job exactly once.
JOBS8 = {"configs3": (8 << 30, 65536, 4), "configs4": (8 << 30, 65536, 2),
         "ragged": ((8 << 30) - 12345, 59460, 3)}


def _fake_sizes(gids):
    return ((gids * 2654435761) >> 7) % 70000 + 1  # (some above 65535: uint32 values)


def _rank8_main(rank, world, port, q):
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        out = {}
        for name, (job, seg, nstreams) in JOBS8.items():
            lay = bd.Layout(job, seg, world, rank, nstreams=nstreams)
            gids = lay.shard.segments
            local = _fake_sizes(gids).to(torch.int32)
            sizes = bd.SizeGather(lay.nseg, world)(local)
            index = bd.frame_index(sizes)
            runs = [(r.gseg, r.lseg, r.count, r.goff, r.loff, r.nbytes) for r in lay.runs]
            parts = [(p.stream, p.lseg, p.count, p.loff, p.nbytes) for p in lay.parts]
            out[name] = (int(sizes.sum()), int(index[-1]), int((index[:-1] * 7 % 1000003).sum()),
                         runs, parts, lay.local_nseg, lay.local_bytes)
        q.put((rank, out))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as ex:  # pragma: no cover - reported to the parent
        q.put((rank, "error: " + repr(ex)))


def test_world8_layout_gather_and_index():
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank8_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r, v in res.items():
        assert not isinstance(v, str), (r, v)
    for name, (job, seg, nstreams) in JOBS8.items():
        nseg = (job + seg - 1) // seg
        ref = _fake_sizes(torch.arange(nseg, dtype=torch.int64))
        ref_index = bd.frame_index(ref)
        want = (int(ref.sum()), int(ref_index[-1]), int((ref_index[:-1] * 7 % 1000003).sum()))
        seg_cover = torch.zeros(nseg, dtype=torch.int32)
        nbytes = 0
        for r in range(world):
            total, last, chk, runs, parts, lnseg, lbytes = res[r][name]
            assert (total, last, chk) == want, (name, r)
            # runs: round-robin batches of 256, stored contiguously in ascending order
            lseg = loff = 0
            for gseg, rl, count, goff, rloff, nb in runs:
                assert (rl, rloff) == (lseg, loff) and gseg % 256 == 0 and (gseg // 256) % world == r
                assert goff == gseg * seg and nb == min(count * seg, job - goff)
                seg_cover[gseg:gseg + count] += 1
                lseg += count
                loff += nb
            assert (lseg, loff) == (lnseg, lbytes)
            nbytes += lbytes
            # parts: nstreams near-equal runs of whole local segments covering the rank's share
            assert sum(p[2] for p in parts) == lnseg and sum(p[4] for p in parts) == lbytes
            assert max(p[2] for p in parts) - min(p[2] for p in parts) <= 1
            assert len(parts) == min(nstreams, lnseg)
        assert bool((seg_cover == 1).all()) and nbytes == job, name
