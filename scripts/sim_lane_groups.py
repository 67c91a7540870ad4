"""Lane-group cursor model (CPU simulation, diagnostic): how many serial decode
steps the slowest lane of a wave needs when each 8x8 block is decoded by L lanes
(L = 1, 2, 4) -- lane 0 from the block's true bit offset, lane k from the bit
position off + k*len/L (speculative; Huffman paths re-synchronise) -- on a real
bitstream. Lane k runs until its path meets lane k+1's (first common symbol
boundary at or beyond lane k+1's start); the last lane runs to the block end.
A block whose lanes never meet falls back to 64 serial steps.

    python scripts/sim_lane_groups.py [--image bigbridge|tile8192|random]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import metalhuffman_amd as mh  # noqa: E402
from metalhuffman_amd import frames as F  # noqa: E402


def windows16(codes: np.ndarray) -> np.ndarray:
    bits = np.unpackbits(codes)
    n = bits.size - 16
    w = np.zeros(n, np.uint32)
    for k in range(16):
        w = (w << 1) | bits[k: k + n]
    return w


def path(width, start, end, max_steps=256):
    """Symbol-start positions from `start` while < end (vectorised over blocks)."""
    P = start.astype(np.int64).copy()
    out = []
    for _ in range(max_steps):
        live = P < end
        if not live.any():
            break
        out.append(np.where(live, P, -1))
        P = np.where(live, P + width[np.minimum(P, width.size - 1)], P)
    return np.stack(out, 1)  # (blocks, steps), -1 past the end


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--image", default="bigbridge", choices=["bigbridge", "tile8192", "random"])
    args = ap.parse_args()
    bb = F.bigbridge()
    img = {"bigbridge": lambda: bb, "tile8192": lambda: F.mirror_tile(bb, 4096, 4096),
           "random": lambda: F.uniform_random(1536, 2048, 1)}[args.image]()
    ef = mh.encode_frame(img)
    t = mh.Huffman.generateLookupTable(ef.canon) if hasattr(mh.Huffman, "generateLookupTable") else None
    from oracle import oracle as O
    single = O.single_table(ef.canon).reshape(65536, 2)
    width_of_window = single[:, 1].astype(np.int64)
    wv = windows16(ef.codes)
    width = width_of_window[wv]
    width[width == 0] = 1  # invalid windows (garbage paths): step 1 bit
    offs = ef.block_offsets.astype(np.int64)
    nb = offs.size
    ends = np.append(offs[1:], offs[-1] + 64 * 16)
    true_path = path(width, offs, ends)  # (nb, 64)
    assert (true_path[:, :64] >= 0).all()
    lens = ends - offs
    res = {}
    for L in (1, 2, 4):
        if L == 1:
            steps = np.full(nb, 64)
        else:
            starts = [offs + (lens * k) // L for k in range(L)]
            paths = [true_path] + [path(width, starts[k], ends) for k in range(1, L)]
            lane_steps = np.zeros((nb, L), np.int64)
            fallback = np.zeros(nb, bool)
            for k in range(L - 1):
                a, b = paths[k], paths[k + 1]
                # first common boundary >= start of lane k+1
                steps_k = np.full(nb, 64)
                for i in range(nb):
                    pa = a[i][a[i] >= 0]
                    pb = set(b[i][b[i] >= 0].tolist())
                    hit = next((n for n, p in enumerate(pa) if p >= starts[k + 1][i] and p in pb), None)
                    if hit is None:
                        fallback[i] = True
                    else:
                        steps_k[i] = hit
                lane_steps[:, k] = steps_k
            lane_steps[:, L - 1] = (paths[L - 1] >= 0).sum(1)
            steps = np.where(fallback, 64, lane_steps.max(1))
            res[f"L{L}_fallback_blocks"] = int(fallback.sum())
        blocks_per_wave = 64 // L
        nw = -(-nb // blocks_per_wave)
        sp = np.zeros(nw * blocks_per_wave, np.int64)
        sp[:nb] = steps
        wave_max = sp.reshape(nw, blocks_per_wave).max(1)
        print(f"L={L}: waves {nw}, block steps mean {steps.mean():.1f}, wave max: p50 {np.median(wave_max):.0f} "
              f"p90 {np.percentile(wave_max, 90):.0f} max {wave_max.max()}; "
              f"sum of wave-max steps {wave_max.sum()} (L=1: {nw * 64 if L == 1 else ''})")
    print(res)


if __name__ == "__main__":
    main()
