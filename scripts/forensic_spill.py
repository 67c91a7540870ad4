"""Round-6 forensics of round 5's silent miscompute.

Decodes frames through the library named by MH_LIB (a variant build) and, where the
raster differs from the input, characterises the error per 8x8 block: which frame,
tile (64 blocks), lane (block in its tile), rows and symbols differ, and the tile's
position in the persistent batch kernel's static schedule (iteration = tile // gstride,
wave = tile % gstride). Prints the first bad blocks' expected and decoded bytes.

Usage (GPU box): MH_LIB=ab/lib_spill.so python scripts/forensic_spill.py [--cases ...]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def block_view(img: np.ndarray) -> np.ndarray:
    h, w = img.shape
    bh, bw = -(-h // 8), -(-w // 8)
    pad = np.zeros((bh * 8, bw * 8), np.uint8)
    pad[:h, :w] = img
    return pad.reshape(bh, 8, bw, 8).transpose(0, 2, 1, 3).reshape(bh * bw, 64)


def main() -> int:
    import torch
    from metalhuffman_amd import codec as C
    from metalhuffman_amd import decoder as D
    from metalhuffman_amd import frames as F

    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="random8192,flatmulti,noesc,general")
    ap.add_argument("--gstride", type=int, default=256 * 3 * 8)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    print("lib", os.environ.get("MH_LIB"), flush=True)
    bb = F.bigbridge()
    for case in args.cases.split(","):
        if case == "random8192":
            imgs = [F.uniform_random(8192, 8192, 1234)]
        elif case == "flatmulti":
            base = F.uniform_random(1024, 1024, 91)
            n = max(1, -(-8400 * 64 // (base.size // 64)))
            imgs = [base] + [F.block_shuffle(base, 500 + s) for s in range(n - 1)]
        elif case == "noesc":
            base = F.mirror_tile(bb, 2048, 8192)
            n = max(1, -(-8400 * 64 // (base.size // 64)))
            imgs = [base] + [F.block_shuffle(base, 500 + s) for s in range(n - 1)]
        else:
            base = np.ascontiguousarray(bb[:1024, :1024])
            n = max(1, -(-8400 * 64 // (base.size // 64)))
            imgs = [base] + [F.block_shuffle(base, 500 + s) for s in range(n - 1)]
        efs = [C.encode_frame(im) for im in imgs]
        t1, t2 = efs[0].tables()
        tabs = D.DeviceTables.upload(t1, t2, dev)
        fr = D.DeviceFrames.pack(efs, dev)
        h, w = imgs[0].shape
        nb = (-(-h // 8)) * (-(-w // 8))
        tpf = -(-nb // 64)
        for rep in range(args.reps):
            out = D.decode(fr, tabs)
            torch.cuda.synchronize(dev)
            got = out[:, :, :w].cpu().numpy()
            nbad_frames = 0
            tiles_bad = []
            lanes = np.zeros(64, np.int64)
            rows = np.zeros(8, np.int64)
            examples = []
            for f, im in enumerate(imgs):
                if np.array_equal(got[f], im):
                    continue
                nbad_frames += 1
                eb, gb = block_view(im), block_view(got[f])
                bad = np.nonzero((eb != gb).any(axis=1))[0]
                for b in bad:
                    tile = f * tpf + b // 64
                    tiles_bad.append(tile)
                    lanes[b % 64] += 1
                    rows += (eb[b].reshape(8, 8) != gb[b].reshape(8, 8)).any(axis=1)
                    if len(examples) < 4:
                        examples.append((f, b, eb[b].copy(), gb[b].copy()))
            tiles_bad = np.unique(np.array(tiles_bad, np.int64))
            print(f"{case} rep {rep}: frames {len(imgs)} bad_frames {nbad_frames} bad_tiles {tiles_bad.size} "
                  f"of {tpf * len(imgs)}", flush=True)
            if tiles_bad.size:
                it = tiles_bad // args.gstride
                print("  tile iterations (tile // gstride) histogram:",
                      dict(zip(*np.unique(it, return_counts=True))), flush=True)
                print("  first bad tiles:", tiles_bad[:16].tolist(), flush=True)
                print("  bad blocks per lane:", lanes.tolist(), flush=True)
                print("  bad rows (count of bad blocks with that row wrong):", rows.tolist(), flush=True)
                for f, b, e, g in examples:
                    d = np.nonzero(e != g)[0]
                    print(f"  frame {f} block {b} (tile {b // 64} lane {b % 64}): first bad symbol {d[0]}, "
                          f"n bad {d.size}", flush=True)
                    print("    want", e.tolist(), flush=True)
                    print("    got ", g.tolist(), flush=True)
                    # does the decoded block equal another block of the frame (stale stage / wrong lane)?
                    eb = block_view(imgs[f])
                    hits = np.nonzero((eb == g).all(axis=1))[0]
                    print("    got equals expected block(s):", hits[:8].tolist(), flush=True)
                    # is it the want shifted by a delta constant (init / prev wrong)?
                    dd = (g.astype(np.int16) - e.astype(np.int16)) % 256
                    print("    got - want (mod 256):", dd.tolist(), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
