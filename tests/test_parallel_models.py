"""CPU models of the wave-parallel reformulations in the entropy coders, checked against the
serial algorithms they replace (the GPU kernels' outputs are checked bit for bit against the
oracle in tests/test_gpu_zstd.py and tests/test_gpu_deflate.py; these tests pin the
decompositions themselves, cheaply, on many more inputs).

1. Huffman code lengths (bitar_amd/csrc/huffman.hip.h): only the two-queue merge is serial
   and it produces the internal weights alone; every node's position in the consumption
   order is a merge rank, its parent the internal node position // 2, depths by pointer
   jumping, then zlib's capping / bl_count repair.  Reference: the oracle's
   bo_huff_lengths (oracle/bitar_deflate_dyn.c), through ctypes.
2. FSE table spread (zstd_compress.hip build_ctable_par, zstd_decompress.hip fse_build):
   the c-th visited position outside the high region takes the symbol whose run of cells
   holds c; each symbol's cells take its state slots in position order.  Reference: the
   serial FSE_buildCTable spread loop (oracle/bitar_zstd.c zs_build_ctable), restated here.
"""
import bisect

import numpy as np
import pytest

import oracle_lib as O


def _huff_model(freq, maxlen):
    f = [int(x) for x in freq]
    nsym = len(f)
    m = sum(1 for x in f if x)
    for s in range(nsym):
        if m >= 2:
            break
        if not f[s]:
            f[s] = 1
            m += 1
    leaf = sorted((s for s in range(nsym) if f[s]), key=lambda s: (f[s], s))
    L = [f[s] for s in leaf]
    # the serial part: internal weights only
    inner, i, j = [], 0, 0
    for t in range(m - 1):
        v = 0
        for _ in range(2):
            if i < m and (j >= t or L[i] <= inner[j]):
                v += L[i]
                i += 1
            else:
                v += inner[j]
                j += 1
        inner.append(v)
    ni, root = m - 1, m - 2
    assert all(inner[k] <= inner[k + 1] for k in range(ni - 1))  # non-decreasing
    # positions by merge rank (leaves first on ties), parents, pointer jumping
    up = [t if t == root else (t + bisect.bisect_right(L, inner[t])) >> 1 for t in range(ni)]
    dep = [0 if t == root else 1 for t in range(ni)]
    span = 1
    while span < ni:
        dep, up = [dep[t] + dep[up[t]] for t in range(ni)], [up[up[t]] for t in range(ni)]
        span <<= 1
    dl = [dep[(k + bisect.bisect_left(inner, L[k])) >> 1] + 1 for k in range(m)]
    over = sum(1 for d in dl if d > maxlen) + sum(1 for t in range(ni - 1) if dep[t] > maxlen)
    bits = [min(d, maxlen) for d in dl]
    if over:
        blc = [0] * 16
        for b in bits:
            blc[b] += 1
        while True:
            b = maxlen - 1
            while blc[b] == 0:
                b -= 1
            blc[b] -= 1
            blc[b + 1] += 2
            blc[maxlen] -= 1
            over -= 2
            if over <= 0:
                break
        cum = 0
        for b in range(maxlen, 0, -1):
            for k in range(cum, cum + blc[b]):
                bits[k] = b
            cum += blc[b]
    lens = np.zeros(nsym, np.uint8)
    for k in range(m):
        lens[leaf[k]] = bits[k]
    return lens


def _huff_cases():
    rng = np.random.default_rng(3)
    fib = [1, 1]
    while len(fib) < 40:
        fib.append(fib[-1] + fib[-2])
    for nsym, ml in ((286, 15), (30, 15), (19, 7), (256, 11)):
        f = np.zeros(nsym, np.uint32)
        k = min(nsym, 30)
        f[:k] = fib[:k]
        yield f, ml
        yield np.zeros(nsym, np.uint32), ml            # no symbol: two padded ones
        g = np.zeros(nsym, np.uint32)
        g[nsym // 2] = 7
        yield g, ml                                     # one symbol
    for t in range(400):
        nsym = int(rng.choice([19, 30, 256, 286]))
        ml = {19: 7, 256: 11}.get(nsym, 15)
        f = np.zeros(nsym, np.uint32)
        k = int(rng.integers(1, nsym + 1))
        idx = rng.choice(nsym, k, replace=False)
        mode = t % 4
        if mode == 0:
            f[idx] = rng.integers(1, 1000, k)
        elif mode == 1:
            f[idx] = (rng.pareto(0.5, k) * 3 + 1).astype(np.uint32)
        elif mode == 2:
            f[idx] = rng.integers(1, 4, k)  # many ties
        else:
            f[idx] = (rng.exponential(1.0, k) ** 4 * 200 + 1).astype(np.uint32)
        yield f, ml


def test_huffman_merge_rank_model_matches_oracle():
    n = 0
    for f, ml in _huff_cases():
        assert np.array_equal(_huff_model(f, ml), O.huff_lengths(f, ml)), (f.tolist(), ml)
        n += 1
    assert n > 400


def _spread_serial(norm, al):
    size, high = 1 << al, (1 << al) - 1
    step, mask = (size >> 1) + (size >> 3) + 3, size - 1
    cells = [None] * size
    for s, v in enumerate(norm):
        if v == -1:
            cells[high] = s
            high -= 1
    pos = 0
    for s, v in enumerate(norm):
        for _ in range(max(v, 0)):
            cells[pos] = s
            pos = (pos + step) & mask
            while pos > high:
                pos = (pos + step) & mask
    assert pos == 0
    # state slots: cell u of symbol s gets cumul[s]++ in position order
    cumul, acc = [], 0
    for v in norm:
        cumul.append(acc)
        acc += 1 if v == -1 else max(v, 0)
    st, nxt = [0] * size, list(cumul)
    for u in range(size):
        st[nxt[cells[u]]] = size + u
        nxt[cells[u]] += 1
    return cells, st


def _spread_parallel(norm, al):
    size = 1 << al
    step, mask = (size >> 1) + (size >> 3) + 3, size - 1
    low = [1 if v == -1 else 0 for v in norm]
    pos = [max(v, 0) for v in norm]
    high = size - 1 - sum(low)
    cum_n = list(np.cumsum([0] + pos[:-1]))
    cells = [None] * size
    seen = 0
    for s, v in enumerate(norm):  # the "less than 1" symbols: top cells, in symbol order
        if v == -1:
            seen += 1
            cells[size - seen] = s
    c = 0
    for k in range(size):
        v = (k * step) & mask
        if v <= high:
            cells[v] = bisect.bisect_right(cum_n, c) - 1  # last run starting at or before c
            c += 1
    assert c == sum(pos)
    cumul = list(np.cumsum([0] + [l + p for l, p in zip(low, pos)][:-1]))
    st, run = [0] * size, [0] * len(norm)
    for u in range(size):  # ranks in position order (the kernel: ballots per 64 cells)
        s = cells[u]
        st[cumul[s] + run[s]] = size + u
        run[s] += 1
    return cells, st


def _normalized(rng, nsym, al):
    """A valid normalized distribution: positive counts and -1 ("less than 1") entries
    summing (|.|) to 2^al, with zeros in between."""
    size = 1 << al
    while True:
        used = rng.random(nsym) < rng.uniform(0.3, 1.0)
        if used.sum() < 2:
            continue
        idx = np.flatnonzero(used)
        nlow = int(rng.integers(0, min(len(idx), 6)))
        low = set(rng.choice(idx, nlow, replace=False).tolist()) if nlow else set()
        rest = [s for s in idx if s not in low]
        budget = size - nlow
        if not rest or budget < len(rest):
            continue
        w = rng.exponential(1.0, len(rest))
        cnt = np.maximum(1, np.floor(w / w.sum() * budget)).astype(int)
        cnt[int(np.argmax(cnt))] += budget - cnt.sum()
        if cnt.min() < 1:
            continue
        norm = [0] * nsym
        for s in low:
            norm[s] = -1
        for s, v in zip(rest, cnt):
            norm[s] = int(v)
        return norm


@pytest.mark.parametrize("al", [5, 6, 8, 9])
def test_fse_spread_rank_model_matches_serial(al):
    rng = np.random.default_rng(al)
    for _ in range(150):
        nsym = int(rng.choice([13, 29, 36, 53]))
        norm = _normalized(rng, nsym, al)
        assert _spread_parallel(norm, al) == _spread_serial(norm, al), norm
