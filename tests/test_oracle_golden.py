"""Pin the oracle (oracle/mh_oracle.c) to the reference's own vectors.

* golden.json was produced by the REAL reference encoder (Shared/HuffmanEncoder.cpp
  compiled unmodified, tests/golden/gen_golden.py): the oracle must reproduce every
  canonical header, code byte and block offset;
* BigBridge T1/T2 SHA-256 recorded in SURVEY.md 8(c) from the reference table builder;
* TEST_6x4_NOT_SQUARE known-answer arrays (Shared/HuffRenderFrame.m:250-300);
* decode(encode(x)) == x through the shader-semantics decoder.
CPU only.
"""
from __future__ import annotations

import hashlib
import os

import numpy as np
import pytest

from helpers import GOLDEN, fibonacci_deltas, golden, image_from_block_deltas


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _canon(d):
    c = np.zeros(256, np.uint8)
    for k, v in d.items():
        c[int(k)] = v
    return c


def test_small_frames_match_reference_encoder(oracle):
    for name, fx in golden()["small_frames"].items():
        img = np.array(fx["pixels"], np.uint8).reshape(fx["height"], fx["width"])
        canon, huff, offs = oracle.encode_frame(img)
        assert np.array_equal(canon, _canon(fx["canon"])), name
        assert huff[:-2].tobytes().hex() == fx["codes_hex"], name   # encoder bytes (+2 renderer pad)
        assert huff[-2:].tolist() == [0, 0]
        assert offs.tolist() == fx["block_offsets"], name
        t1, t2 = oracle.split_tables(canon)
        out = oracle.decode_frame_shader(offs, huff, t1, t2, fx["width"], fx["height"])
        assert np.array_equal(out, img), name


def test_survey_known_answers(oracle):
    """4x4 ramp and 8x8 ident code bytes."""
    g = golden()["small_frames"]
    assert g["TEST_4x4_INCREASING1"]["codes_hex"].startswith("59787d65d1fd9706acb60000")
    assert g["TEST_8x8_IDENT"]["codes_hex"].startswith("f264e4c9f4c9c993264e4c9f4c9c99000000")


def test_kat_6x4_not_square(oracle):
    """HuffRenderFrame.m:250-300: 2x2 blocks, no deltas -> root offsets, widths, windows."""
    k = golden()["kat_6x4"]
    img = np.array(k["pixels"], np.uint8).reshape(4, 6)
    sym = oracle.split_blocks(img, bdim=2)
    canon, codes, offs = oracle.huffman_encode(sym, stride=4)
    assert codes.tobytes().hex() == k["ref_codes_hex"] == "e2983f2ef5903a800000"
    assert offs.tolist() == k["ref_block_offsets"] == [0, 10, 18, 29, 40, 48]
    t1, t2 = oracle.split_tables(canon)
    buf = np.concatenate([codes, np.zeros(2, np.uint8)])
    dec, bitpos = oracle.decode_from_tables(t1, t2, sym.size, buf, want_offsets=True)
    assert np.array_equal(dec, sym)
    # expectations are per pixel in raster order; pixel (x, y) is symbol
    # (y%2)*2 + x%2 of block (y//2)*3 + x//2
    for y in range(4):
        for x in range(6):
            i = ((y // 2) * 3 + x // 2) * 4 + (y % 2) * 2 + (x % 2)
            r = y * 6 + x
            root = offs[i // 4]
            assert root == k["root_bit_offset"][r]
            assert bitpos[i] - root == k["current_bit_offset"][r]
            assert canon[sym[i]] == k["bit_width"][r]
            p = int(bitpos[i])
            b = [int(v) for v in buf[p // 8: p // 8 + 3]]
            m = p % 8
            win = ((((b[0] << m) & 0xFF) << 8) | (b[1] << m) | (b[2] >> (8 - m))) & 0xFFFF
            assert win == k["bit_pattern"][r]


@pytest.mark.parametrize("wl", ["bigbridge", "bigbridge_crop_777x1001", "random_1024_seed1234",
                                "bigbridge_shuffle_seed7", "image_png_L_256", "image_png_L_512",
                                "tile_8192"])
def test_workload_hashes(oracle, bigbridge, wl):
    from metalhuffman_amd import frames as F
    rec = golden()["workloads"][wl]
    if wl == "bigbridge":
        img = bigbridge
    elif wl == "bigbridge_crop_777x1001":
        img = F.crop(bigbridge, 1001, 777)
    elif wl == "random_1024_seed1234":
        img = F.uniform_random(1024, 1024, 1234)
    elif wl == "bigbridge_shuffle_seed7":
        img = F.block_shuffle(bigbridge, 7)
    elif wl == "tile_8192":
        img = F.mirror_tile(bigbridge, 8192, 8192)
    else:
        from PIL import Image
        gray = np.array(Image.open(os.path.join(GOLDEN, "Image.png")).convert("L"), np.uint8)
        img = gray if wl.endswith("512") else np.ascontiguousarray(gray[:256, :256])
    assert sha(img) == rec["input_sha256"]
    canon, huff, offs = oracle.encode_frame(img)
    assert sha(canon) == rec["canon_sha256"]
    assert sha(huff) == rec["huffbuff_sha256"]
    assert sha(offs.astype("<u4")) == rec["offsets_sha256"]
    if "t1_sha256" in rec:
        t1, t2 = oracle.split_tables(canon)
        assert sha(t1) == rec["t1_sha256"] and sha(t2) == rec["t2_sha256"]
        assert t2.size == rec["t2_bytes"]


def test_bigbridge_roundtrip_and_both_cpu_decoders(oracle, bigbridge):
    canon, huff, offs = oracle.encode_frame(bigbridge)
    t1, t2 = oracle.split_tables(canon)
    out = oracle.decode_frame_shader(offs, huff, t1, t2, 2048, 1536)
    assert np.array_equal(out, bigbridge)
    nsym = offs.size * 64
    a = oracle.decode_from_tables(t1, t2, nsym, huff)
    b = oracle.decode_single_table(oracle.single_table(canon), nsym, huff)
    assert np.array_equal(a, b)


def test_code_too_long_is_rejected(oracle):
    d = fibonacci_deltas(18, 64 * 64 * 2, seed=1)  # depth 17 -> the reference asserts
    rc, canon = oracle.code_lengths(d)
    assert rc == -2 and canon.max() == 17


def test_odd_sizes_roundtrip(oracle, bigbridge):
    for h, w in [(1, 1), (3, 5), (9, 17), (1001, 777), (8, 4096)]:
        img = np.ascontiguousarray(np.tile(bigbridge, (1, 2))[:h, :w])
        canon, huff, offs = oracle.encode_frame(img)
        t1, t2 = oracle.split_tables(canon)
        assert np.array_equal(oracle.decode_frame_shader(offs, huff, t1, t2, w, h), img)


@pytest.mark.ref
@pytest.mark.skipif(not os.path.isdir("/root/reference/Shared"), reason="needs /root/reference")
def test_oracle_matches_reference_encoder_random_histograms(oracle):
    """Tie-breaking stress: many small alphabets with repeated frequencies."""
    assert oracle.build_ref()
    r = np.random.default_rng(11)
    for trial in range(40):
        nsym = int(r.integers(1, 40))
        alphabet = r.choice(256, size=nsym, replace=False).astype(np.uint8)
        weights = r.integers(1, 6, size=nsym) ** r.integers(1, 4)
        d = r.choice(alphabet, size=64 * int(r.integers(1, 50)), p=weights / weights.sum())
        rc, _ = oracle.code_lengths(d)
        if rc != 0:
            continue
        c1, k1, o1 = oracle.huffman_encode(d, 64)
        c2, k2, o2 = oracle.ref_encode(d, 64)
        assert np.array_equal(c1, c2) and np.array_equal(k1, k2) and np.array_equal(o1, o2), trial


def test_block_deltas_helper_roundtrip(oracle):
    d = fibonacci_deltas(12, 64 * 64 * 4, seed=2)
    img = image_from_block_deltas(d, 128, 128)
    blocks = oracle.split_blocks(img)
    for b in range(blocks.size // 64):
        blocks[b * 64:(b + 1) * 64] = oracle.delta_encode(blocks[b * 64:(b + 1) * 64])
    assert np.array_equal(blocks, d)


def test_cpu_baseline_pipeline_rasters(oracle, mh):
    """bench.py's CPU pipeline leg (decode + undelta + raster) reproduces the frames
    it times, on 3 threads over 5 frames of a partial-block crop."""
    from metalhuffman_amd import frames as F
    base = np.ascontiguousarray(F.bigbridge()[:203, :517])
    imgs = [base] + [np.ascontiguousarray(np.roll(base, 37 * k, axis=1)) for k in range(1, 5)]
    pairs = [(mh.encode_frame(im), im) for im in imgs]
    pairs = [p for p in pairs if np.array_equal(p[0].canon, pairs[0][0].canon)]
    efs, imgs = [p[0] for p in pairs], [p[1] for p in pairs]
    t1, t2 = efs[0].tables()
    ras = [np.zeros((203, 517), np.uint8) for _ in efs]
    sec = oracle.time_decode_pipeline(t1, t2, 517, 203, [ef.codes for ef in efs], 3, reps=2, rasters=ras)
    assert sec > 0
    for r, im in zip(ras, imgs):
        assert np.array_equal(r, im)
