"""Step model of the round-3 lane-pair kernel (mh_decode.hip lp_decode; CPU simulation,
diagnostic): lane A decodes from the block start, lane B from the middle bit M until the
block end; B's starts in [M, M + 64) form its window mask, which reaches A at the first
checkpoint step (n = 8, 12, 16, ...) after the mask is final (B past M + 64 or stopped).
A stops at the first of its starts that is one of B's -- at that step once it holds the
mask, or at the checkpoint if it had already passed one; A decodes the whole block when
it leaves the window unmatched; a block whose B decoded too few symbols is finished by A
(repair). Prints per-lane steps, the wave's loop length (its slowest lane, 32 blocks)
and the per-step exchange counts, for comparison with the PMC instruction counts.

    python scripts/sim_lane_pairs_ckpt.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import metalhuffman_amd as mh  # noqa: E402
from metalhuffman_amd import frames as F  # noqa: E402
from oracle import oracle as O  # noqa: E402

ef = mh.encode_frame(F.bigbridge())
W = O.single_table(ef.canon).reshape(65536, 2)[:, 1].astype(np.int64)
bits = np.unpackbits(ef.codes)
n = bits.size - 16
win = np.zeros(n, np.int64)
for k in range(16):
    win = (win << 1) | bits[k:k + n]
width = W[win]
offs = ef.block_offsets.astype(np.int64)
nb = offs.size
ends = np.append(offs[1:], offs[-1])
lens = ends - offs
mid = offs + lens // 2
spec = np.arange(nb) + 1 < nb
spec &= (lens >= 32) & (lens <= 1024)


def path(start, steps=64):
    P = np.empty((start.size, steps + 1), np.int64)
    P[:, 0] = start
    for s in range(steps):
        P[:, s + 1] = P[:, s] + width[np.minimum(P[:, s], width.size - 1)]
    return P


WIN = int(os.environ.get("WIN", "128"))  # window bits (the kernel: 128)
A = path(offs)            # A's starts: A[:, k] = start of symbol k (true path)
B = path(mid)             # B's starts from the middle
stepsA = np.full(nb, 64)
stepsB = np.zeros(nb, np.int64)
overshoot = np.zeros(nb, np.int64)
repair = 0
for i in range(nb):
    if not spec[i]:
        continue
    # B: decodes until its start >= end (or 64 symbols)
    bs = B[i]
    nB = int(np.argmax(bs >= ends[i])) if (bs >= ends[i]).any() else 64
    nB = min(nB, 64)
    stepsB[i] = nB
    inwin = (bs[:nB] - mid[i] >= 0) & (bs[:nB] - mid[i] < WIN)
    mB = set((bs[:nB][inwin] - mid[i]).tolist())
    # B's mask final at the step after which its cursor >= M + 64, or when B stops
    past = np.nonzero(bs[:nB + 1] - mid[i] >= WIN)[0]
    t_fin = min(int(past[0]) if past.size else nB, nB)
    # first checkpoint >= t_fin at which A can receive it (checks run before step n)
    ck = max(8, ((t_fin + 3) // 4) * 4)
    a = A[i]
    rel = a - mid[i]
    meet = None
    for k in range(64):
        if 0 <= rel[k] < WIN and rel[k] in mB:
            meet = k
            break
        if rel[k] >= WIN:
            break
    if meet is None:
        stepsA[i] = 64
        continue
    ia = meet
    jb = sum(1 for r in mB if r < rel[meet])
    if nB < jb + 64 - ia:
        repair += 1
        stepsA[i] = 64
        continue
    stepsA[i] = max(meet, ck) if meet < ck else meet
    overshoot[i] = max(0, ck - meet)
lane_max = np.maximum(stepsA, stepsB)
pad = (-nb) % 32
wm = np.concatenate([lane_max, np.zeros(pad, np.int64)]).reshape(-1, 32).max(1)
print(f"blocks {nb}, speculated {spec.sum()}, repaired {repair}")
print(f"A steps mean {stepsA.mean():.1f}  B steps mean {stepsB.mean():.1f}  A overshoot mean {overshoot.mean():.2f}")
print(f"block max-lane steps mean {lane_max.mean():.1f} p50 {np.median(lane_max):.0f} p99 {np.percentile(lane_max, 99):.0f}")
print(f"wave loop length (32 blocks): p50 {np.median(wm):.0f} p90 {np.percentile(wm, 90):.0f} "
      f"p99 {np.percentile(wm, 99):.0f} max {wm.max()}  (default kernel: 64 on every wave)")
print(f"lane-steps per block: {(stepsA + stepsB).mean():.1f} (default 64)")
print(f"blocks where A decodes all 64: {(stepsA == 64).mean() * 100:.2f} %")
print(f"wave loop length mean {wm.mean():.1f} over {wm.size} waves")
