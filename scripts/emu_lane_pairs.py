"""Bit-level emulation of lp_decode (mh_decode.hip, lane-pair kernel) on the CPU
(diagnostic): every block's two lanes step in lock-step exactly as the kernel's
unrolled loop does (checkpoints, window masks, meeting point, repair, row assembly
with the delta rebase) and the assembled bytes are compared with the oracle's decode.

    python scripts/emu_lane_pairs.py [n_blocks]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import metalhuffman_amd as mh  # noqa: E402
from metalhuffman_amd import frames as F  # noqa: E402
from oracle import oracle as O  # noqa: E402

WIN = 128


def emulate(ef, nmax):
    single = O.single_table(ef.canon).reshape(65536, 2).astype(np.int64)
    bits = np.unpackbits(np.concatenate([ef.codes, np.zeros(256, np.uint8)]))
    n = bits.size - 16
    win = np.zeros(n, np.int64)
    for k in range(16):
        win = (win << 1) | bits[k:k + n]
    sym, wid = single[win, 0].tolist(), single[win, 1].tolist()
    offs = [int(x) for x in ef.block_offsets]
    nb = len(offs)
    init = ef.block_init if ef.block_init is not None else np.zeros(nb, np.uint8)
    delta = not (ef.flags & 1)
    fbits = ef.codes.size * 8
    out = np.zeros((min(nb, nmax), 64), np.uint8)
    stats = dict(met=0, rep=0, alone=0)
    for b in range(min(nb, nmax)):
        exact = b + 1 < nb
        end = offs[b + 1] if exact else min(fbits, offs[b] + 1024)
        ln = end - offs[b]
        mid = offs[b] + ln // 2
        spec = exact and 32 <= ln <= 1024
        lanes = []
        for is_b in (False, True):
            lanes.append(dict(pos=mid if is_b else offs[b], S=0 if is_b else int(init[b]),
                              act=(not is_b) or spec, chk=spec and not is_b, have=False,
                              mine=0, other=0, nd=0, srel=WIN, o=[0] * 64))
        A, B = lanes

        def step(L, k):
            p = L["pos"]
            L["S"] = (L["S"] + sym[p]) & 0xFF if delta else L["S"]
            L["o"][k] = L["S"] if delta else sym[p]
            L["pos"] = p + wid[p]

        for k in range(64):
            if not (A["act"] or B["act"]):
                break
            if k >= 8 and k % 4 == 0 and A["chk"] and not A["have"]:
                fin = (not B["act"]) or B["pos"] - mid >= WIN
                if fin:
                    A["have"] = True
                    A["other"] = B["mine"]
                    cm = A["mine"] & A["other"]
                    if cm:
                        A["chk"] = A["act"] = False
                        A["srel"] = (cm & -cm).bit_length() - 1
                    elif A["pos"] - mid >= WIN:
                        A["chk"] = False
            for L, is_b in ((A, False), (B, True)):
                if not L["act"]:
                    continue
                rel = L["pos"] - mid
                if 0 <= rel < WIN:
                    if L["chk"] and L["have"] and (L["other"] >> rel) & 1:
                        L["chk"] = L["act"] = False
                        L["srel"] = rel
                        continue
                    L["mine"] |= 1 << rel
                elif L["chk"] and L["have"] and rel >= WIN:
                    L["chk"] = False
                step(L, k)
                L["nd"] = k + 1
                if (is_b and L["pos"] >= end) or k == 63:
                    L["act"] = False
        met = A["srel"] < WIN
        ia, jb = 64, 0
        if met:
            s = A["srel"]
            ia = A["nd"] - bin(A["mine"] >> s).count("1")
            jb = bin(A["other"] & ((1 << s) - 1)).count("1")
        ok = met and B["nd"] >= jb + 64 - ia
        if met and not ok:
            stats["rep"] += 1
            for k in range(A["nd"], 64):
                step(A, k)
        if ok:
            stats["met"] += 1
        elif not met:
            stats["alone"] += 1
        if not ok:
            ia, jb = 64, 0
        pa = A["o"][ia - 1] if ia else int(init[b])
        pb = B["o"][jb - 1] if jb else 0
        cadd = (pa - pb) & 0xFF if delta else 0
        out[b] = [A["o"][i] if i < ia else (B["o"][i - ia + jb] + cadd) & 0xFF for i in range(64)]
    return out, stats


def oracle_blocks(ef):
    t1, t2 = ef.tables()
    img = O.decode_frame_shader(ef.block_offsets, ef.codes, t1, t2, ef.width, ef.height,
                                block_init=ef.block_init, delta=not (ef.flags & 1))
    bw, bh = (ef.width + 7) // 8, (ef.height + 7) // 8
    pad = np.zeros((bh * 8, bw * 8), np.uint8)
    pad[:ef.height, :ef.width] = img
    return pad.reshape(bh, 8, bw, 8).transpose(0, 2, 1, 3).reshape(-1, 64), img


if __name__ == "__main__":
    nmax = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    bb = F.bigbridge()
    cases = [("bigbridge", mh.encode_frame(bb)),
             ("init_zero_delta", mh.encode_frame(np.ascontiguousarray(bb[:768, :1024]), init_zero_delta=True)),
             ("no_delta_random", mh.encode_frame(F.uniform_random(512, 256, 9), flags=mh.MH_FLAG_NO_DELTA))]
    ef = mh.encode_frame(np.ascontiguousarray(bb[:768, :1024]))
    from metalhuffman_amd import codec as C
    junk = np.random.default_rng(5).integers(0, 256, size=ef.codes.size, dtype=np.uint8)
    cases.append(("junk", C.EncodedFrame(ef.width, ef.height, ef.canon, junk, ef.block_offsets, None, ef.flags)))
    for name, e in cases:
        got, st = emulate(e, nmax)
        ref, _ = oracle_blocks(e)
        bad = int((got != ref[:got.shape[0]]).any(1).sum())
        print(f"{name:16s} blocks {got.shape[0]} mismatched {bad} {st}")
