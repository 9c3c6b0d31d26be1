"""GPU tests of the sharded job (bitar_amd.job.ShardedJob): BASELINE configs[3] at full
size on one GPU -- an 8 GiB Arrow record-batch job of 64 KiB chunks, round-robin batches,
four concurrent queue-pair streams -- with a byte-exact round trip, a frame index spanning
the job, and sampled chunks bit-exact against the oracle; plus the offset generator the
ranks use to materialise only their batches."""
import numpy as np
import pytest

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
        for g in (0, 255, 256, 32767, 32768, 65537, 131071):  # part boundaries included
            plain = down(job.data[g * seg:(g + 1) * seg])
            r, comp = O.lz4_compress(plain.tobytes())
            assert r == 0 and len(comp) == sizes[g], g
            got = down(job.slab[g * job.stride:g * job.stride + int(sizes[g])]).tobytes()
            assert got == comp, g
        job.free()
    finally:
        e.close()


def test_zstd_column_8gib_configs4():
    """BASELINE configs[4] at its full 8 GiB job size on one GPU: level-1-class Zstd frames
    per 64 KiB chunk of an int64 column buffer (kind 5, the Parquet-column shape), dealt in
    round-robin batches over two queue-pair streams, byte-exact round trip, the job-wide frame
    index, and sampled chunks bit-exact against the oracle's encoder."""
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
        for g in (0, 255, 256, 65535, 65536, 131071):
            plain = down(job.data[g * seg:(g + 1) * seg])
            r, comp = O.zstd_compress(plain.tobytes())
            assert r == 0 and len(comp) == sizes[g], g
            got = down(job.slab[g * job.stride:g * job.stride + int(sizes[g])]).tobytes()
            assert got == comp, g
        job.free()
    finally:
        e.close()
