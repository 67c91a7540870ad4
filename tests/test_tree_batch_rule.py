"""The GPU encoder's batched Huffman merge (enc_tree_kernel, mh_encode.hip) restated
in Python and checked against the host codec's serial tree (mh_code_lengths, which
follows the reference's sorted node array, HuffmanEncoder.cpp:29-145): the same code
lengths for every histogram, including tie-heavy and error (depth > 16) ones, and
the round counts the kernel relies on for valid codes."""
from __future__ import annotations

import ctypes

import numpy as np


def batched_lengths(f):
    """Rounds of up to 32 merges: with Q the merge of both queues (a leaf first on a
    tie), the next k merges pair Q[0..2k) in order while Q[2k-1] <= Q[0] + Q[1]."""
    leaves = sorted((int(f[s]), s) for s in range(256) if f[s])
    n = len(leaves)
    out = [0] * 256
    if n == 1:
        out[leaves[0][1]] = 1
        return out, 0
    lw = [w for w, _ in leaves]
    iw, par = [], {}
    li = ii = m = rounds = 0
    while m < n - 1:
        q, a, b = [], li, ii
        while len(q) < 64 and (a < n or b < len(iw)):
            if a < n and (b >= len(iw) or lw[a] <= iw[b]):
                q.append((lw[a], a))
                a += 1
            else:
                q.append((iw[b], n + b))
                b += 1
        s0 = q[0][0] + q[1][0]
        k = 0
        while k < 32 and 2 * k + 1 < len(q) and q[2 * k + 1][0] <= s0:
            k += 1
        k = min(k, n - 1 - m)
        nl = sum(1 for _, node in q[: 2 * k] if node < n)
        base = len(iw)
        for t in range(k):
            iw.append(q[2 * t][0] + q[2 * t + 1][0])
            par[q[2 * t][1]] = par[q[2 * t + 1][1]] = n + base + t
        li, ii, m, rounds = li + nl, ii + 2 * k - nl, m + k, rounds + 1
    root = 2 * n - 2
    for i in range(n):
        d, x = 0, i
        while x != root:
            x, d = par[x], d + 1
        out[leaves[i][1]] = min(d, 255)
    return out, rounds


def _host_lengths(f):
    from metalhuffman_amd import _native as N
    h = (ctypes.c_uint8 * 256)()
    rc = N.lib().mh_code_lengths(np.ascontiguousarray(f, np.uint64).ctypes.data_as(N._u64p), h)
    return list(h), rc


def test_batched_merge_equals_serial_tree():
    rng = np.random.default_rng(11)
    for t in range(600):
        k = int(rng.integers(2, 257))
        syms = rng.choice(256, k, replace=False)
        f = np.zeros(256, np.uint64)
        mode = t % 5
        if mode == 0:
            f[syms] = rng.integers(1, 5, k)
        elif mode == 1:
            f[syms] = rng.integers(1, 1_000_000, k)
        elif mode == 2:
            f[syms] = 7
        elif mode == 3:
            fib = [1, 1]
            while len(fib) < k:
                fib.append(min(fib[-1] + fib[-2], 2 ** 31))
            f[syms] = np.array(fib[:k], np.uint64)
        else:
            f[syms] = np.round(2.0 ** rng.uniform(0, 20, k)).astype(np.uint64)
        got, _ = batched_lengths(f)
        want, _ = _host_lengths(f)
        assert got == want, t


def test_valid_codes_need_few_rounds():
    import metalhuffman_amd as mh
    from metalhuffman_amd import frames as F
    img = F.bigbridge()
    blk = mh.split_blocks(img).reshape(-1, 64).astype(np.int16)
    f = np.bincount((np.diff(blk, axis=1, prepend=0) & 0xFF).ravel(), minlength=256).astype(np.uint64)
    got, rounds = batched_lengths(f)
    assert got == _host_lengths(f)[0]
    assert rounds <= 20          # 255 serial merges in 15 rounds
