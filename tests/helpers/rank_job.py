"""A rank of the CPU rehearsal of the sharded job (tests/test_launch.py): started by the
real launcher (bitar_amd.launch.spawn), it lays out its share with bitar_amd.dist.Layout,
compresses every part with the oracle (standing in for the rank's GPU: test plumbing), and
runs the real size all-gather (SizeGather over gloo) and frame index.  Writes its view of
the job to <outdir>/rank<r>.json."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import oracle_lib as O  # noqa: E402
from bitar_amd import dist as bd  # noqa: E402
from bitar_amd import launch  # noqa: E402


def main():
    outdir, job_bytes, seg, nstreams, batch = (sys.argv[1], int(sys.argv[2]), int(sys.argv[3]),
                                               int(sys.argv[4]), int(sys.argv[5]))
    world, rank, local = launch.rank_env()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    L = bd.Layout(job_bytes, seg, world, rank, nstreams, batch)
    whole = O.fill(O.KIND_MIXED, 5, job_bytes)
    local_data = np.concatenate([whole[r.goff:r.goff + r.nbytes] for r in L.runs]) \
        if L.runs else np.zeros(0, np.uint8)
    assert local_data.size == L.local_bytes
    sizes = np.zeros(L.local_nseg, np.uint32)
    blobs = {}
    for p in L.parts:  # one "launch" per queue-pair stream
        part = local_data[p.loff:p.loff + p.nbytes]
        for k in range(p.count):
            s = part[k * seg:(k + 1) * seg].tobytes()
            r, c = O.lz4_compress(s)
            assert r == 0
            sizes[p.lseg + k] = len(c)
            blobs[p.lseg + k] = c
    g = bd.SizeGather(L.nseg, world, batch)
    gsizes = g(torch.from_numpy(sizes.view(np.int32)))
    index = bd.frame_index(gsizes)
    # this rank's frames at their global positions
    segs = L.shard.segments.tolist()
    frames = {int(gid): blobs[j].hex() for j, gid in enumerate(segs)}
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump({"rank": rank, "world": world, "local": local,
                   "sizes": gsizes.tolist(), "index": index.tolist(), "frames": frames,
                   "parts": [(p.stream, p.lseg, p.count) for p in L.parts],
                   "master": os.environ["MASTER_ADDR"]}, f)
    dist.barrier()
    dist.destroy_process_group()
    if rank == 1 and os.environ.get("RANK_JOB_FAIL") == "1":
        sys.exit(3)


if __name__ == "__main__":
    main()
