"""CPU rehearsal of the multi-GPU path: the real launcher (bitar_amd.launch.spawn, what
`bench.py --gpus N` uses) starts world-size-2 and -3 rank processes that shard a job with the
real layout (bitar_amd.dist.Layout: round-robin batches, parts per stream) and run the real
size all-gather + frame index over gloo; every rank must hold the same global sizes and
index as a single-process compression of the whole job, and the frames of all ranks, placed
by the index, must decode back to the job."""
import json
import os
import sys

import numpy as np
import pytest

import oracle_lib as O
from bitar_amd import dist as bd
from bitar_amd import launch

HELPER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "helpers", "rank_job.py")


@pytest.mark.parametrize("world,nstreams", [(2, 2), (3, 1)])
def test_launcher_runs_sharded_job(tmp_path, world, nstreams):
    seg, batch = 4096, 3
    job = 29 * seg + 777  # 30 segments, ragged tail, 10 batches
    rc = launch.spawn(world, HELPER, [str(tmp_path), str(job), str(seg), str(nstreams),
                                      str(batch)], timeout=240)
    assert rc == 0
    ranks = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    data = O.fill(O.KIND_MIXED, 5, job)
    nseg = (job + seg - 1) // seg
    ref = []
    for g in range(nseg):
        r, c = O.lz4_compress(data[g * seg:(g + 1) * seg].tobytes())
        assert r == 0
        ref.append(c)
    ref_sizes = [len(c) for c in ref]
    ref_index = [0] + list(np.cumsum(ref_sizes))
    image = bytearray(ref_index[-1])
    seen = set()
    for r in ranks:
        assert r["world"] == world and r["master"] == "127.0.0.1"
        assert r["sizes"] == ref_sizes
        assert r["index"] == ref_index
        for gid, hx in r["frames"].items():
            gid = int(gid)
            assert gid not in seen
            seen.add(gid)
            image[ref_index[gid]:ref_index[gid + 1]] = bytes.fromhex(hx)
    assert seen == set(range(nseg))
    assert bytes(image) == b"".join(ref)
    # parts: whole segments, one per stream, covering the rank's share
    for r in ranks:
        L = bd.Layout(job, seg, world, r["rank"], nstreams, batch)
        assert [tuple(p) for p in r["parts"]] == [(p.stream, p.lseg, p.count) for p in L.parts]
        assert sum(p.count for p in L.parts) == L.local_nseg


def test_launcher_reports_a_failed_rank(tmp_path):
    seg = 4096
    rc = launch.spawn(2, HELPER, [str(tmp_path), str(8 * seg), str(seg), "1", "2"],
                      extra_env={"RANK_JOB_FAIL": "1"}, timeout=240)
    assert rc == 3


def test_layout_properties():
    for job, seg, world, ns, batch in ((1 << 30, 65536, 8, 4, 256), (8 << 30, 65536, 3, 4, 256),
                                       (100, 7, 2, 3, 5), (0, 64, 2, 2, 4), (65536, 65536, 4, 2, 256)):
        nseg = (job + seg - 1) // seg
        got = []
        total = 0
        for r in range(world):
            L = bd.Layout(job, seg, world, r, ns, batch)
            assert L.nseg == nseg
            ids = []
            for run in L.runs:
                ids += list(range(run.gseg, run.gseg + run.count))
                assert run.goff == run.gseg * seg
            assert ids == L.shard.segments.tolist()
            got += ids
            total += L.local_bytes
            assert sum(p.nbytes for p in L.parts) == L.local_bytes
            counts = [p.count for p in L.parts]
            assert not counts or max(counts) - min(counts) <= 1
        assert sorted(got) == list(range(nseg))
        assert total == job
    # weak scaling: N GiB over N ranks -> exactly 1 GiB each
    for world in (1, 2, 4, 8):
        for r in range(world):
            assert bd.Layout(world << 30, 65536, world, r).local_bytes == 1 << 30


def test_rank_env_defaults(monkeypatch):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    assert launch.rank_env() == (1, 0, 0)
    assert not launch.is_rank_process()


def test_bench_parent_spawns_without_touching_gpu():
    """bench.py's parent branch imports neither torch nor HIP before spawning."""
    src = open(os.path.join(os.path.dirname(HELPER), "..", "..", "bench.py")).read()
    m = src.index("def main():")
    head = src[m:src.index("import torch\n", m)]
    assert "launch.spawn(args.gpus" in head and "torch" not in head.replace("torch.distributed.run", "")
