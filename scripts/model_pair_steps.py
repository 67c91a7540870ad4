"""Step model of a two-symbol lookup for the single-frame kernel (CPU, diagnostic, round 5).

A lane looks up a K-bit window; the entry holds one symbol, or two when both codes fit in
the K bits. A wave's loop runs until its slowest lane has 64 symbols, so its length is the
max over its 64 lanes of that lane's lookups. Prints the distribution of wave loop lengths
against the 64 of the one-symbol step, for the bench's config-2 frames (block-shuffled
BigBridge), the natural frame and the 8192^2 tile's first rows.

    python scripts/model_pair_steps.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import metalhuffman_amd as mh  # noqa: E402
from metalhuffman_amd import frames as F  # noqa: E402
from oracle import oracle as O  # noqa: E402


def lookups(ef, K: int) -> np.ndarray:
    """Per block: lookups to decode its 64 symbols with a K-bit pair table."""
    W = O.single_table(ef.canon).reshape(65536, 2)[:, 1].astype(np.int64)  # code length per 16-bit window
    bits = np.unpackbits(np.concatenate([ef.codes, np.zeros(8, np.uint8)]))
    n = bits.size - 16
    win = np.zeros(n, np.int64)
    for k in range(16):
        win = (win << 1) | bits[k:k + n]
    width = W[win]
    offs = ef.block_offsets.astype(np.int64)
    nb = offs.size
    pos = offs.copy()
    cnt = np.zeros(nb, np.int64)
    steps = np.zeros(nb, np.int64)
    live = np.ones(nb, bool)
    while live.any():
        p = np.minimum(pos, n - 1)
        l1 = width[p]
        p2 = np.minimum(pos + l1, n - 1)
        l2 = width[p2]
        pair = (l1 + l2 <= K) & (cnt + 2 <= 64)
        adv = np.where(pair, l1 + l2, l1)
        pos = np.where(live, pos + adv, pos)
        cnt = np.where(live, cnt + np.where(pair, 2, 1), cnt)
        steps += live
        live = cnt < 64
    return steps


def report(name: str, ef, K: int) -> None:
    s = lookups(ef, K)
    pad = (-s.size) % 64
    wm = np.concatenate([s, np.zeros(pad, np.int64)]).reshape(-1, 64).max(1)
    print(f"{name:34s} K={K}: lane lookups mean {s.mean():5.1f} | wave loop p50 {np.median(wm):3.0f} "
          f"p90 {np.percentile(wm, 90):3.0f} max {wm.max():3d} mean {wm.mean():5.1f} (one-symbol step: 64)")


bb = F.bigbridge()
frames = [("bigbridge shuffles (bench config 2)", mh.encode_frame(F.block_shuffle(bb, 1))),
          ("bigbridge (natural)", mh.encode_frame(bb)),
          ("crop 777x1001", mh.encode_frame(np.ascontiguousarray(bb[100:1101, 200:977])))]
for K in (13, 14):
    for name, ef in frames:
        report(name, ef, K)
