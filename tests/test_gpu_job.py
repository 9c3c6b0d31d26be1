"""GPU tests of the sharded job (bitar_amd.job.ShardedJob): BASELINE configs[3] at full
size on one GPU -- an 8 GiB Arrow record-batch job of 64 KiB chunks, round-robin batches,
four concurrent queue-pair streams -- with a byte-exact round trip, a frame index spanning
the job, and EVERY chunk bit-exact against the oracle (tests/gpu_parity.py); plus the offset
generator the ranks use to materialise only their batches."""
import numpy as np
import pytest

import gpu_parity as P
import oracle_lib as O
from test_gpu_lz4 import down, eng  # noqa: F401  (fixture reuse)

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.mark.parametrize("kind", [1, 2, 6])
@pytest.mark.parametrize("off,n", [(0, 1000), (64, 4096 + 3), ((1 << 20) - 64, 3 << 20),
                                   (3 << 20, 65536)])
def test_fill_at_offset_matches_oracle(eng, kind, off, n):
    d = eng.empty(n)
    eng.fill(kind, 99, d, n=n, offset=off)
    assert np.array_equal(down(d), O.fill(kind, 99, off + n)[off:])


def test_recordbatch_8gib_four_streams():
    import bitar_amd
    from bitar_amd.job import ShardedJob
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    e = bitar_amd.Engine(0, num_streams=4)
    try:
        seg = 65536
        job = ShardedJob(e, bitar_amd.CODEC_LZ4, 8 << 30, seg, world=1, rank=0, nstreams=4)
        assert len(job.layout.parts) == 4 and job.layout.local_nseg == 131072
        job.generate(2, 3)
        for _ in range(2):  # twice: the second step reuses every buffer
            job.step()
        job.sync()
        assert job.verify()
        sizes = down(job.sizes).astype(np.uint32)
        assert int(job.index[-1].item()) == int(sizes.astype(np.int64).sum())
        assert np.array_equal(np.diff(down(job.index)), sizes.astype(np.int64))
        # every one of the 131072 chunks (all four parts, their boundaries included)
        P.assert_every_segment_matches_oracle(bitar_amd.CODEC_LZ4, job.data, 8 << 30, seg,
                                              job.slab, job.stride, job.sizes)
        job.free()
    finally:
        e.close()


def test_zstd_column_8gib_configs4():
    """BASELINE configs[4] at its full 8 GiB job size on one GPU: level-1-class Zstd frames
    per 64 KiB chunk of an int64 column buffer (kind 5, the Parquet-column shape), dealt in
    round-robin batches over two queue-pair streams, byte-exact round trip, the job-wide frame
    index, and every chunk bit-exact against the oracle's encoder."""
    import bitar_amd
    from bitar_amd.job import ShardedJob
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    e = bitar_amd.Engine(0, num_streams=2)
    try:
        seg = 65536
        job = ShardedJob(e, bitar_amd.CODEC_ZSTD, 8 << 30, seg, world=1, rank=0, nstreams=2)
        assert job.layout.local_nseg == 131072
        job.generate(5, 11)
        job.step()
        job.sync()
        assert job.verify()
        sizes = down(job.sizes).astype(np.uint32)
        assert int(job.index[-1].item()) == int(sizes.astype(np.int64).sum())
        assert sizes.astype(np.int64).sum() < (8 << 30) // 3  # a column compresses > 3x
        P.assert_every_segment_matches_oracle(bitar_amd.CODEC_ZSTD, job.data, 8 << 30, seg,
                                              job.slab, job.stride, job.sizes)
        job.free()
    finally:
        e.close()
