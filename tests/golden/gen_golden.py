"""Generate tests/golden/golden.json from the REAL reference encoder.

Run in the build container only (needs /root/reference):
    python tests/golden/gen_golden.py

What it records (all data, no reference source):
  * small hand-written frames of Shared/HuffRenderFrame.m:135-460 and the
    TEST_6x4_NOT_SQUARE known-answer arrays (:250-300);
  * for each workload: SHA-256 of the canonical header, codes and block offsets the
    reference encoder (Shared/HuffmanEncoder.cpp, compiled unmodified by
    oracle/Makefile into oracle/_ref/ref_encode) emits for the renderer's producer
    step (8x8 zero-padded blocks, per-block deltas, AAPLRenderer.m:374-688);
  * BigBridge T1/T2 SHA-256 as recorded in SURVEY.md 8(c) (reference table builder,
    HuffmanUtil.cpp:338-667, built in the survey session).
The huffBuff hashes include the renderer's 2 extra zero bytes (AAPLRenderer.m:576-585).
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

REF_SHARED = "/root/reference/Shared"


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# Shared/HuffRenderFrame.m:135-460 (pixel values, raster order)
SMALL = {
    "TEST_4x4_INCREASING1": (4, 4, [0, 1, 4, 5, 2, 3, 6, 7, 8, 9, 12, 13, 10, 11, 14, 15]),
    "TEST_4x4_INCREASING2": (4, 4, [0, 1, 4, 0, 2, 3, 5, 0, 6, 7, 10, 0, 8, 9, 11, 0]),
    "TEST_4x8_INCREASING1": (4, 8, [0, 1, 4, 5, 2, 3, 6, 7, 8, 9, 12, 13, 10, 11, 14, 15,
                                    0, 1, 4, 5, 2, 3, 6, 7, 8, 8, 10, 10, 9, 9, 10, 10]),
    "TEST_2x8_INCREASING1": (2, 8, list(range(16))),
    "TEST_6x4_NOT_SQUARE": (6, 4, [0, 1, 2, 3, 4, 5, 3, 3, 1, 1, 2, 2, 5, 4, 3, 2, 1, 0, 2, 2, 1, 1, 3, 3]),
    "TEST_8x8_IDENT": (8, 8, [0, 1, 4, 5, 10, 11, 14, 15, 2, 3, 6, 7, 12, 13, 16, 17,
                              8, 9, 12, 13, 18, 19, 22, 23, 10, 11, 14, 15, 20, 21, 24, 25,
                              30, 31, 34, 35, 40, 41, 44, 45, 32, 33, 36, 37, 42, 43, 46, 47,
                              38, 39, 42, 43, 48, 49, 52, 53, 40, 41, 44, 45, 50, 51, 54, 55]),
}
_r16x8 = []
for y in range(8):
    _r16x8 += [8 * (y % 4) + x for x in range(8)] + [2, 4, 6, 8, 10, 12, 14, 16]
SMALL["TEST_16x8_IDENT"] = (16, 8, _r16x8)
_a = [0, 1, 2, 3, 4, 5, 6, 7]
_b = [10, 9, 8, 7, 6, 5, 4, 3]
_c = [102, 104, 106, 108, 110, 112, 114, 116]
_d = [50, 51, 52, 53, 54, 55, 56, 57]
_e = [58, 57, 56, 55, 54, 53, 52, 51]
_f = [3, 5, 6, 3, 1, 2, 1, 1]
_top = (_a + _c) + (_b + _c) + (_a + _c) + (_b + _c)
_bot = (_d + _f) + (_e + _f) + (_d + _f) + (_e + _f)
SMALL["TEST_16x16_IDENT"] = (16, 16, _top + _bot + _top + _bot)
_row0 = [228, 228, 228, 44, 2] + [0] * 11
SMALL["TEST_16x16_IDENT2"] = (16, 16, _row0 + [0] * 240)
SMALL["TEST_16x16_IDENT3"] = (16, 16, [0] * 128 + _row0 + [0] * 112)

# TEST_6x4_NOT_SQUARE debug expectations (HuffRenderFrame.m:250-300): 2x2 blocks,
# no deltas; per pixel (raster order) root bit offset, bit width, 16-bit window.
KAT_6x4 = {
    "block_dim": 2,
    "root_bit_offset": [0, 0, 10, 10, 18, 18, 0, 0, 10, 10, 18, 18,
                        29, 29, 40, 40, 48, 48, 29, 29, 40, 40, 48, 48],
    "current_bit_offset": [0, 4, 0, 2, 0, 4, 6, 8, 4, 6, 7, 9,
                           0, 3, 0, 2, 0, 2, 7, 9, 4, 6, 6, 8],
    "bit_width": [4, 2, 2, 2, 4, 3, 2, 2, 2, 2, 2, 2, 3, 4, 2, 2, 2, 4, 2, 2, 2, 2, 2, 2],
    "bit_pattern": [0xE298, 0x2983, 0x60FC, 0x83F2, 0xFCBB, 0xCBBD,
                    0xA60F, 0x983F, 0x0FCB, 0x3F2E, 0x5DEB, 0x77AC,
                    0xDEB2, 0xF590, 0x903A, 0x40EA, 0x3A80, 0xEA00,
                    0x5903, 0x640E, 0x03A8, 0x0EA0, 0xA000, 0x8000],
}

# BigBridge outputs of the reference table builder.
BIGBRIDGE_T1 = "9c7b1fabf94689e77b38bb1ce751bb3c0b2d4aa93771ef4a2f07165bde493fa4"
BIGBRIDGE_T2 = "a01cfa9bae0fbd5bdae28ada06ba4c7cb83c15fa9ebdcda91e6adeeb830f6f51"


def producer_symbols(img: np.ndarray, block_dim: int = 8, delta: bool = True) -> np.ndarray:
    blocks = O.split_blocks(img, bdim=block_dim)
    if delta:
        bs = block_dim * block_dim
        for b in range(blocks.size // bs):
            blocks[b * bs:(b + 1) * bs] = O.delta_encode(blocks[b * bs:(b + 1) * bs])
    return blocks


def ref_record(img: np.ndarray) -> dict:
    sym = producer_symbols(img)
    canon, codes, offs = O.ref_encode(sym, 64)
    huff = np.concatenate([codes, np.zeros(2, np.uint8)])
    return {
        "width": int(img.shape[1]), "height": int(img.shape[0]),
        "input_sha256": sha(img), "canon_sha256": sha(canon), "huffbuff_sha256": sha(huff),
        "offsets_sha256": sha(offs.astype("<u4")), "huffbuff_bytes": int(huff.size),
        "max_code_len": int(canon.max()),
        "bits_per_symbol": float((codes.size - 2) * 8 / sym.size),
    }


def main() -> int:
    if not os.path.isdir(REF_SHARED):
        print("needs /root/reference (build container only)", file=sys.stderr)
        return 1
    O.build()
    O.build_ref()
    for asset in ("BigBridge.png", "Image.png"):
        dst = os.path.join(HERE, asset)
        if not os.path.exists(dst):
            shutil.copy(os.path.join(REF_SHARED, asset), dst)
    from metalhuffman_amd import frames as F
    from PIL import Image

    out: dict = {"generator": "tests/golden/gen_golden.py", "small_frames": {}, "workloads": {}}
    for name, (w, h, px) in SMALL.items():
        img = np.array(px, np.uint8).reshape(h, w)
        sym = producer_symbols(img)
        canon, codes, offs, header = O.ref_encode(sym, 64, with_header=True)
        out["small_frames"][name] = {
            "width": w, "height": h, "pixels": px,
            "canon": {str(i): int(c) for i, c in enumerate(canon) if c},
            "codes_hex": codes.tobytes().hex(), "block_offsets": offs.tolist(),
            "container_header_hex": header.tobytes().hex(),
        }
    img6 = np.array(SMALL["TEST_6x4_NOT_SQUARE"][2], np.uint8).reshape(4, 6)
    sym6 = producer_symbols(img6, block_dim=2, delta=False)
    c6, k6, o6 = O.ref_encode(sym6, 4)
    kat = dict(KAT_6x4)
    kat.update({"pixels": SMALL["TEST_6x4_NOT_SQUARE"][2], "width": 6, "height": 4,
                "ref_canon": {str(i): int(c) for i, c in enumerate(c6) if c},
                "ref_codes_hex": k6.tobytes().hex(), "ref_block_offsets": o6.tolist()})
    out["kat_6x4"] = kat

    bb = F.bigbridge()
    rec = ref_record(bb)
    rec.update({"t1_sha256": BIGBRIDGE_T1, "t2_sha256": BIGBRIDGE_T2, "t2_bytes": 14848})
    out["workloads"]["bigbridge"] = rec
    out["workloads"]["bigbridge_crop_777x1001"] = ref_record(F.crop(bb, 1001, 777))
    out["workloads"]["random_1024_seed1234"] = ref_record(F.uniform_random(1024, 1024, 1234))
    out["workloads"]["bigbridge_shuffle_seed7"] = ref_record(F.block_shuffle(bb, 7))
    out["workloads"]["tile_8192"] = ref_record(F.mirror_tile(bb, 8192, 8192))
    gray = np.array(Image.open(os.path.join(HERE, "Image.png")).convert("L"), np.uint8)
    out["workloads"]["image_png_L_512"] = ref_record(gray)
    out["workloads"]["image_png_L_256"] = ref_record(np.ascontiguousarray(gray[:256, :256]))

    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", os.path.join(HERE, "golden.json"))
    return 0


if __name__ == "__main__":
    sys.exit(main())
