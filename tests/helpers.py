"""Shared helpers for the test suite (CPU and GPU)."""
from __future__ import annotations

import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden() -> dict:
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


def image_from_block_deltas(deltas: np.ndarray, width: int, height: int) -> np.ndarray:
    """Integrate per-block deltas (block order, 64 per block) into a raster whose
    producer step (split + per-block delta) yields exactly `deltas`.
    width and height must be multiples of 8 (no pad region to reproduce)."""
    assert width % 8 == 0 and height % 8 == 0
    bw, bh = width // 8, height // 8
    d = deltas.reshape(bh * bw, 64).astype(np.uint16)
    vals = (np.cumsum(d, axis=1) & 0xFF).astype(np.uint8)
    return np.ascontiguousarray(vals.reshape(bh, bw, 8, 8).transpose(0, 2, 1, 3).reshape(height, width))


def fibonacci_deltas(n_symbols: int, total: int, seed: int = 0) -> np.ndarray:
    """A delta stream whose histogram is Fibonacci-shaped over `n_symbols` symbols
    (deepest code = n_symbols - 1 bits), shuffled."""
    fib = [1, 1]
    while len(fib) < n_symbols:
        fib.append(fib[-1] + fib[-2])
    fib = np.array(fib[:n_symbols], dtype=np.int64)
    reps = max(1, total // int(fib.sum()))
    counts = fib * reps
    syms = np.repeat(np.arange(n_symbols, dtype=np.uint8)[::-1], counts)
    out = np.zeros(total, np.uint8)
    out[: min(total, syms.size)] = syms[:total]
    np.random.default_rng(seed).shuffle(out)
    return out


def long_span_deltas(width: int, height: int, seed: int = 0) -> np.ndarray:
    """Mostly-zero deltas with every rare symbol packed into the FIRST tile
    (64 blocks): that tile's code span exceeds the kernel's LDS window and takes the
    global-memory path, while every code stays <= 16 bits."""
    nb = (width // 8) * (height // 8)
    d = np.zeros(nb * 64, np.uint8)
    r = np.random.default_rng(seed)
    first = 64 * 64
    rare = r.integers(1, 256, size=first, dtype=np.uint8)
    d[:first] = rare
    return d


def lane_pair_oversize_deltas(seed: int = 0) -> np.ndarray:
    """512x512 deltas whose first 32 blocks hold 249 rare symbols x 8 (15-bit codes under
    a geometric chain of 7 common symbols): that 32-block lane-pair tile spans 3,735 B,
    more than round 2's 3,712-B lane-pair stage, with codes above 14 bits
    (the 13-bit table with escapes)."""
    n = 512 * 512
    r = np.random.default_rng(seed)
    rare = np.repeat(np.arange(7, 256, dtype=np.uint8), 8)
    head = np.zeros(2048, np.uint8)
    head[: rare.size] = rare
    r.shuffle(head)
    rest = np.repeat(np.arange(7, dtype=np.uint8), [n >> (k + 1) for k in range(7)])[: n - 2048]
    rest = np.concatenate([rest, np.zeros(n - 2048 - rest.size, np.uint8)])
    r.shuffle(rest)
    return np.concatenate([head, rest])


def refill_extreme_deltas(n_symbols: int, width: int, height: int, seed: int = 0) -> np.ndarray:
    """Deltas with a Fibonacci histogram over `n_symbols` symbols (deepest code
    n_symbols - 1 bits) rearranged so that many blocks hold a prefix of p short codes
    (p = 0..32, every bit alignment of the cursor) followed by a run of the LONGEST codes:
    the decoders' refill points then see the cursor at its deepest (sh up to 47 bits into
    the 64-bit window). The histogram, hence the code lengths, is unchanged."""
    nb = (width // 8) * (height // 8)
    d = fibonacci_deltas(n_symbols, nb * 64, seed=seed)
    vals, counts = np.unique(d, return_counts=True)
    order = np.argsort(counts, kind="stable")          # rarest (longest code) first
    rare = np.concatenate([np.full(counts[i], vals[i], np.uint8) for i in order])
    common = int(vals[order[-1]])                      # the 1-bit code
    out = np.empty(nb * 64, np.uint8)
    r_i = 0
    pool = []
    for b in range(nb):
        p = b % 33
        blk = np.full(64, common, np.uint8)
        take = min(64 - p, rare.size - r_i)
        blk[p:p + take] = rare[r_i:r_i + take]
        r_i += take
        out[b * 64:(b + 1) * 64] = blk
    # the histogram must match the Fibonacci one: the loop above used at most the rare
    # symbols once each; top up / trim the common symbol so the multiset is d's
    want = np.bincount(d, minlength=256)
    have = np.bincount(out, minlength=256)
    diff = want[common] - have[common]
    if diff < 0:  # too many common symbols: put the unused rare ones back in their place
        left = rare[r_i:]
        idx = np.nonzero(out == common)[0][-left.size:] if left.size else np.array([], np.int64)
        out[idx] = left
        pool = left
    assert np.array_equal(np.bincount(out, minlength=256), want), "histogram changed"
    return out
