"""CPU tests of the C-ABI boundary: the library builds, loads, and exports every symbol
include/bitar_hip.h declares.  No compute calls (no GPU here)."""
import ctypes
import os
import re

import bitar_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    with open(os.path.join(ROOT, "include", "bitar_hip.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(bitar_hip_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    if not os.path.exists(bitar_amd.LIB_PATH):
        bitar_amd.build()
    L = ctypes.CDLL(bitar_amd.LIB_PATH)
    declared = header_symbols()
    assert len(declared) >= 19
    for name in declared:
        assert hasattr(L, name), name
    assert sorted(bitar_amd.ABI_SYMBOLS) == declared


def test_abi_version_and_slot_sizes():
    L = bitar_amd.lib()
    assert L.bitar_hip_abi_version() == 3
    # LZ4_compressBound(65536) = 65809 -> 256-B rounded slot
    assert bitar_amd.slot_size(bitar_amd.CODEC_LZ4, 65536) == 66048
    assert bitar_amd.slot_size(bitar_amd.CODEC_LZ4, 59460) >= 59460 + 59460 // 255 + 16
    assert bitar_amd.slot_size(bitar_amd.CODEC_DEFLATE, 59460) >= (59460 * 9 + 7) // 8 + 16
    assert bitar_amd.slot_size(99, 100) == 0


def test_encoder_reach():
    """bitar_hip_max_distance: the encoders' match-distance cap, which the oracle restates
    (BO_MAX_DIST / the wide parse's cap) and the front-end reports as its window."""
    B = bitar_amd
    for c in (B.CODEC_LZ4, B.CODEC_DEFLATE, B.CODEC_DEFLATE_DYNAMIC, B.CODEC_ZSTD):
        assert B.max_distance(c) == 2560
    assert B.max_distance(B.CODEC_LZ4_WIDE) == 14848
    assert B.max_distance(99) == 0


def test_no_device_is_not_an_error_for_count():
    # in the build container there is no GPU: the count is 0, not a crash
    n = bitar_amd.device_count()
    assert n >= 0
