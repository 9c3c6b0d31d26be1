"""Loader for the committed golden vectors (tests/golden/manifest.json + golden.bin)."""
import hashlib
import json
import os

import numpy as np

import oracle_lib

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def manifest():
    with open(os.path.join(GOLDEN_DIR, "manifest.json")) as f:
        return json.load(f)


def blob_file():
    with open(os.path.join(GOLDEN_DIR, "golden.bin"), "rb") as f:
        return f.read()


def vectors(codec=None):
    """Yield (entry, compressed_bytes, expected_plain_bytes)."""
    m = manifest()
    data = blob_file()
    plain_cache = {}
    for e in m["entries"]:
        if codec is not None and e["codec"] != codec:
            continue
        inp = m["inputs"][e["input"]]
        key = e["input"]
        if key not in plain_cache:
            plain_cache[key] = oracle_lib.fill(inp["kind"], inp["seed"], inp["n"]).tobytes()
            assert hashlib.sha256(plain_cache[key]).hexdigest() == inp["sha256"], key
        blob = data[e["offset"]:e["offset"] + e["size"]]
        assert hashlib.sha256(blob).hexdigest() == e["blob_sha256"]
        yield e, blob, plain_cache[key]


def as_u8(b):
    return np.frombuffer(b, dtype=np.uint8).copy()
