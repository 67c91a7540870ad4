"""LDS bank-conflict model of the batch kernel's table gathers on a real bitstream
(CPU simulation, diagnostic). For every tile (64 blocks = 64 lanes) and decode
step, the lanes' next-window table addresses are banked per MI355X_MICROARCH.md
(ds_read_b32/u16: two 32-lane groups, bank = (byte_addr / 4) % 32, one LDS cycle per
distinct dword on the busiest bank, identical dwords broadcast). Compares the
13-bit single-level table with a small first level + masked second-level gather
for the lanes whose code is longer than the first level.

    python scripts/sim_lds_banks.py [--tiles N]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import metalhuffman_amd as mh  # noqa: E402
from metalhuffman_amd import frames as F  # noqa: E402


def group_cycles(dw, active):
    """dw: (steps, 32) dword addresses, active: bool mask -> LDS cycles per step."""
    out = np.zeros(dw.shape[0])
    for s in range(dw.shape[0]):
        a = dw[s][active[s]]
        if a.size == 0:
            continue
        u = np.unique(a)
        out[s] = np.bincount(u % 32, minlength=32).max()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", type=int, default=96)
    ap.add_argument("--image", default="bigbridge", choices=["bigbridge", "tile8192"])
    args = ap.parse_args()
    img = F.bigbridge() if args.image == "bigbridge" else F.mirror_tile(F.bigbridge(), 8192, 8192)
    ef = mh.encode_frame(img)
    canon = ef.canon.astype(np.int64)
    bits = np.unpackbits(ef.codes)
    nb = ef.n_blocks
    offs = ef.block_offsets.astype(np.int64)
    t1, t2 = ef.tables()
    t1 = t1.view(np.uint8).reshape(-1, 2)
    t2 = t2.view(np.uint8).reshape(-1, 2)
    rng = np.random.default_rng(0)
    tiles = rng.choice(nb // 64, size=min(args.tiles, nb // 64), replace=False)
    res = {}
    for k1 in (13, 8, 9, 10, 11):
        res[k1] = []
    for t in tiles:
        pos = offs[t * 64:(t + 1) * 64].copy()
        idx13 = np.zeros((64, 64), np.int64)
        lens = np.zeros((64, 64), np.int64)
        for j in range(64):
            # 16-bit window at each lane's cursor
            w = np.zeros(64, np.int64)
            for b in range(16):
                w = (w << 1) | bits[pos + b]
            e = t1[w >> 8]
            sym, ln = e[:, 0].astype(np.int64), e[:, 1].astype(np.int64)
            esc = ln == 0
            if esc.any():
                e2 = t2[sym[esc] * 256 + (w[esc] & 0xFF)]
                ln[esc] = e2[:, 1]
            idx13[:, j] = w >> 3
            lens[:, j] = ln
            pos += ln
        for k1 in (13, 8, 9, 10, 11):
            if k1 == 13:
                dw = (idx13.T >> 1)  # u16 entries, 2 per dword
                act = np.ones_like(dw, bool)
                c = sum(group_cycles(dw[:, g * 32:(g + 1) * 32], act[:, g * 32:(g + 1) * 32]) for g in (0, 1))
            else:
                i1 = idx13.T >> (13 - k1)
                c = sum(group_cycles((i1 >> 1)[:, g * 32:(g + 1) * 32], np.ones((64, 32), bool)) for g in (0, 1))
                esc = lens.T > k1
                dw2 = (idx13.T >> 1) + 100000
                c2 = sum(group_cycles(dw2[:, g * 32:(g + 1) * 32], esc[:, g * 32:(g + 1) * 32]) for g in (0, 1))
                res.setdefault(f"{k1}esc", []).append(esc.any(axis=1).mean())
                res.setdefault(f"{k1}lanes", []).append(esc.mean())
                c = c + c2
            res[k1].append(c.mean())
    print(f"{args.image}: {len(tiles)} tiles; LDS cycles per wave-gather (2 groups; 2 = conflict-free)")
    for k in (13, 8, 9, 10, 11):
        extra = ""
        if k != 13:
            extra = (f"  (steps with an escape gather {np.mean(res[f'{k}esc']) * 100:.1f} %, "
                     f"lanes escaping {np.mean(res[f'{k}lanes']) * 100:.1f} %)")
        print(f"  first level {k:2d} bits: {np.mean(res[k]):.2f}{extra}")


if __name__ == "__main__":
    main()


def pair_model(image="bigbridge", ntiles=48, bits_l1=13):
    """Two symbols per step: one gather in a 2^bits_l1-entry table of u32 pair entries
    (both symbols when len1 + len2 <= bits_l1), plus a masked gather of the second
    symbol for the lanes whose pair does not fit."""
    img = F.bigbridge() if image == "bigbridge" else F.mirror_tile(F.bigbridge(), 8192, 8192)
    ef = mh.encode_frame(img)
    bits = np.unpackbits(ef.codes)
    offs = ef.block_offsets.astype(np.int64)
    t1, t2 = ef.tables()
    t1 = t1.view(np.uint8).reshape(-1, 2)
    t2 = t2.view(np.uint8).reshape(-1, 2)
    nb = ef.n_blocks
    rng = np.random.default_rng(0)
    tiles = rng.choice(nb // 64, size=min(ntiles, nb // 64), replace=False)
    cyc, fb_steps, fb_lanes = [], [], []
    for t in tiles:
        pos = offs[t * 64:(t + 1) * 64].copy()
        wins, lens = [], []
        for j in range(64):
            w = np.zeros(64, np.int64)
            for b in range(16):
                w = (w << 1) | bits[pos + b]
            e = t1[w >> 8]
            sym, ln = e[:, 0].astype(np.int64), e[:, 1].astype(np.int64)
            esc = ln == 0
            if esc.any():
                ln[esc] = t2[sym[esc] * 256 + (w[esc] & 0xFF)][:, 1]
            wins.append(w >> (16 - bits_l1))
            lens.append(ln.copy())
            pos += ln
        wins, lens = np.array(wins), np.array(lens)  # (64 steps, 64 lanes)
        for s in range(0, 64, 2):
            dw = wins[s]  # u32 entries: one dword each
            c = sum(group_cycles(dw[None, g * 32:(g + 1) * 32], np.ones((1, 32), bool))[0] for g in (0, 1))
            fb = lens[s] + lens[s + 1] > bits_l1
            dw2 = wins[s + 1]
            c2 = sum(group_cycles(dw2[None, g * 32:(g + 1) * 32], fb[None, g * 32:(g + 1) * 32])[0] for g in (0, 1))
            cyc.append(c + c2)
            fb_steps.append(fb.any())
            fb_lanes.append(fb.mean())
    print(f"{image}: pair table {bits_l1} bits: LDS cycles per 2-symbol step {np.mean(cyc):.2f} "
          f"(vs 2 x single gather); fallback in {np.mean(fb_steps) * 100:.1f} % of steps, "
          f"{np.mean(fb_lanes) * 100:.1f} % of lanes")
