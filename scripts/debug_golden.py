#!/usr/bin/env python3
"""Decode every golden vector of one codec on the GPU one at a time; report failures."""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tests"))
import golden_lib  # noqa: E402
import oracle_lib as O  # noqa: E402
from test_gpu_lz4 import _decode_blobs  # noqa: E402


def main():
    import bitar_amd
    codec = sys.argv[1] if len(sys.argv) > 1 else "lz4"
    eng = bitar_amd.Engine(0)
    c = O.CODEC_LZ4 if codec == "lz4" else O.CODEC_DEFLATE
    bad = 0
    for e, blob, plain in golden_lib.vectors(codec):
        ok, out, prod = _decode_blobs(eng, c, [blob], 65536)
        if not ok or prod[0] != len(plain) or out[:len(plain)].tobytes() != plain:
            bad += 1
            first = next((i for i in range(min(len(plain), int(prod[0]) if ok else 0))
                          if out[i] != plain[i]), None)
            print("FAIL", e["producer"], e["input"], "ok", ok, "prod", int(prod[0]),
                  "want", len(plain), "first_diff", first)
    print("bad", bad)


if __name__ == "__main__":
    main()
