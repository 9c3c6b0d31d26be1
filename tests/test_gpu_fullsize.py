"""Parity at BASELINE sizes, every segment: the whole 1 GiB call of each codec leg is compared
with the oracle's encoder segment by segment (sizes and every slot byte), round-trips
byte-exactly through our decoders, and every GPU frame of a multi-kind call decodes with the
stock library (zlib raw inflate, liblz4 LZ4_decompress_safe, libzstd ZSTD_decompress).
Reference contract: the round trip of apps/demo_app.cc:534-543, 671-686 and the per-op
failure rule of src/device.cc:512-520."""
import numpy as np
import pytest

import gpu_parity as P
import oracle_lib as O
import stock_lib as S
from test_gpu_lz4 import eng  # noqa: F401  (fixture reuse)

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

# (codec name, input kind, segment size): configs[2] LZ4 (and its ratio point), configs[4]'s
# codec on the Arrow record batch, the reference's own DEFLATE frame (FIXED and DYNAMIC)
LEGS = [("LZ4", 1, 65536), ("LZ4_WIDE", 1, 65536), ("ZSTD", 2, 65536),
        ("DEFLATE", 1, 59460), ("DEFLATE_DYNAMIC", 1, 59460)]


@pytest.mark.parametrize("name,kind,seg", LEGS, ids=[l[0] for l in LEGS])
def test_every_segment_1gib_vs_oracle(eng, name, kind, seg):
    import bitar_amd
    codec = getattr(bitar_amd, "CODEC_" + name)
    n = 1 << 30
    data = eng.empty(n)
    eng.fill(kind, 0, data)
    slab, stride, sizes = eng.compress(codec, data, seg)
    out, prod = eng.decompress(codec, slab, stride, sizes, seg)
    eng.sync()
    assert torch.equal(out[:n], data)
    del out
    nseg = (n + seg - 1) // seg
    gs = P.assert_every_segment_matches_oracle(codec, data, n, seg, slab, stride, sizes)
    assert gs.size == nseg
    print(f"{name}: {nseg} segments bit-exact, ratio {n / gs.astype(np.int64).sum():.4f}")
    del data, slab, sizes
    torch.cuda.empty_cache()


STOCK = {"LZ4": S.LZ4, "LZ4_WIDE": S.LZ4, "ZSTD": S.ZSTD, "DEFLATE": S.DEFLATE,
         "DEFLATE_DYNAMIC": S.DEFLATE}


@pytest.mark.parametrize("name", list(STOCK))
def test_stock_decodes_every_frame_of_a_multikind_call(eng, name):
    """160 MiB: 32 MiB regions of random, Silesia-style, record-batch, int64-column and log
    input in one call; the stock library decodes every frame to the input."""
    import bitar_amd
    codec = getattr(bitar_amd, "CODEC_" + name)
    seg = 59460 if name.startswith("DEFLATE") else 65536
    region = 32 << 20
    kinds = (0, 1, 2, 5, 6)
    n = region * len(kinds)
    data = eng.empty(n)
    for j, k in enumerate(kinds):
        eng.fill(k, 40 + j, data[j * region:(j + 1) * region])
    slab, stride, sizes = eng.compress(codec, data, seg)
    eng.sync()
    P.stock_decodes_every_frame(STOCK[name], slab, stride, sizes, data, n, seg)
