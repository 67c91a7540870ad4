"""GPU parity: the HIP decoder vs the oracle and the reference encoder's fixtures.

Every case is bit-exact (integer/byte work). Inputs are produced by the product's
host codec (itself byte-identical to the reference encoder, test_codec_parity.py)
or taken verbatim from the reference encoder's output (golden.json), so these
tests show the decoder consuming the reference's buffers unchanged.
"""
from __future__ import annotations

import numpy as np
import pytest

from helpers import (fibonacci_deltas, golden, image_from_block_deltas, long_span_deltas,
                     refill_extreme_deltas)

pytestmark = pytest.mark.gpu


def _decode(frames_list, device, prepared=True, flags_override=None):
    from metalhuffman_amd import decoder as D
    t1, t2 = frames_list[0].tables()
    tabs = D.DeviceTables.upload(t1, t2, device, prepare_lut=prepared)
    fr = D.DeviceFrames.pack(frames_list, device)
    out = D.decode(fr, tabs)
    import torch
    torch.cuda.synchronize(device)
    return out[..., : fr.width].cpu().numpy()


def _oracle_decode(O, ef):
    t1, t2 = ef.tables()
    return O.decode_frame_shader(ef.block_offsets, ef.codes, t1, t2, ef.width, ef.height,
                                 block_init=ef.block_init, delta=not (ef.flags & 1))


@pytest.mark.parametrize("prepared", [True, False])
def test_bigbridge_bit_exact(mh, oracle, device, bigbridge, prepared):
    ef = mh.encode_frame(bigbridge)
    out = _decode([ef], device, prepared)[0]
    assert np.array_equal(out, bigbridge)
    assert np.array_equal(out, _oracle_decode(oracle, ef))


def test_reference_encoder_small_frames(mh, device):
    """Buffers exactly as the reference encoder emitted them (golden.json)."""
    from metalhuffman_amd import codec as C
    for name, fx in golden()["small_frames"].items():
        w, h = fx["width"], fx["height"]
        canon = np.zeros(256, np.uint8)
        for k, v in fx["canon"].items():
            canon[int(k)] = v
        codes = np.frombuffer(bytes.fromhex(fx["codes_hex"]), np.uint8)
        huff = np.concatenate([codes, np.zeros(2, np.uint8)])  # AAPLRenderer.m:576-585
        ef = C.EncodedFrame(w, h, canon, huff, np.array(fx["block_offsets"], np.uint32))
        out = _decode([ef], device)[0]
        assert np.array_equal(out, np.array(fx["pixels"], np.uint8).reshape(h, w)), name


@pytest.mark.parametrize("hw", [(1, 1), (7, 9), (9, 7), (8, 8), (1001, 777), (5, 2051), (4097, 13),
                                (64, 520), (3, 65535)])
def test_odd_sizes(mh, oracle, device, bigbridge, hw):
    h, w = hw
    tile = np.tile(bigbridge, (max(1, -(-h // bigbridge.shape[0])), max(1, -(-w // bigbridge.shape[1]))))
    img = np.ascontiguousarray(tile[:h, :w])
    ef = mh.encode_frame(img)
    out = _decode([ef], device)[0]
    assert np.array_equal(out, img)
    if h * w <= 4_000_000:
        assert np.array_equal(out, _oracle_decode(oracle, ef))


def test_uniform_random(mh, oracle, device):
    from metalhuffman_amd import frames as F
    img = F.uniform_random(1024, 1024, 1234)
    ef = mh.encode_frame(img)
    assert ef.canon.max() == 8
    out = _decode([ef], device)[0]
    assert np.array_equal(out, img)


def test_batch_block_shuffled(mh, device, bigbridge):
    from metalhuffman_amd import frames as F
    imgs = [F.block_shuffle(bigbridge, s) for s in range(16)]
    efs = [mh.encode_frame(im) for im in imgs]
    out = _decode(efs, device)
    for i, im in enumerate(imgs):
        assert np.array_equal(out[i], im), i


def _decode_repeat(efs, device, reps):
    import torch
    from metalhuffman_amd import decoder as D
    t1, t2 = efs[0].tables()
    tabs = D.DeviceTables.upload(t1, t2, device)
    fr = D.DeviceFrames.pack(efs, device)
    outs = []
    for _ in range(reps):
        out = D.decode(fr, tabs)
        torch.cuda.synchronize(device)
        outs.append(out[..., : fr.width].cpu().numpy())
    return outs


def test_multi_tile_waves_repeat(mh, device, bigbridge):
    """Several tiles per wave (the pipelined loop's steady state), launched repeatedly
    on the same buffers: every launch decodes every tile exactly once."""
    from metalhuffman_amd import frames as F
    imgs = [F.block_shuffle(bigbridge, 100 + s) for s in range(24)]
    efs = [mh.encode_frame(im) for im in imgs]
    for out in _decode_repeat(efs, device, 3):
        for i, im in enumerate(imgs):
            assert np.array_equal(out[i], im), i


def test_oversize_tiles_in_multi_tile_waves(mh, oracle, device):
    """Tiles leave the pipelined loop for the slow path while waves hold several tiles."""
    d = long_span_deltas(1024, 256)
    img = image_from_block_deltas(d, 1024, 256)
    ef = mh.encode_frame(img)
    for out in _decode_repeat([ef] * 200, device, 2):  # 12,800 tiles
        for i in range(200):
            assert np.array_equal(out[i], img), i


@pytest.mark.parametrize("n_sym", [14, 15, 17])
def test_long_codes_delta(mh, oracle, device, n_sym):
    """Fibonacci histograms: codes up to 16 bits, exercising the second LDS level."""
    d = fibonacci_deltas(n_sym, 512 * 512, seed=n_sym)
    img = image_from_block_deltas(d, 512, 512)
    ef = mh.encode_frame(img)
    assert ef.canon.max() == n_sym - 1
    out = _decode([ef], device)[0]
    assert np.array_equal(out, img)
    assert np.array_equal(out, _oracle_decode(oracle, ef))


def test_no_delta_mode(mh, oracle, device):
    """IMPL_DELTAS_BEFORE_HUFF_ENCODING off: symbols are the pixels themselves."""
    d = fibonacci_deltas(17, 256 * 256, seed=3)
    img = d.reshape(256, 256)
    ef = mh.encode_frame(img, flags=mh.MH_FLAG_NO_DELTA)
    assert ef.canon.max() == 16
    out = _decode([ef], device)[0]
    assert np.array_equal(out, img)
    assert np.array_equal(out, _oracle_decode(oracle, ef))


def test_init_zero_delta_mode(mh, oracle, device, bigbridge):
    """IMPL_DELTAS_AND_INIT_ZERO_DELTA_BEFORE_HUFF_ENCODING: per-block init byte."""
    img = np.ascontiguousarray(bigbridge[:768, :1024])  # (512x640 would need a 17-bit code)
    ef = mh.encode_frame(img, init_zero_delta=True)
    assert ef.block_init is not None
    out = _decode([ef], device)[0]
    assert np.array_equal(out, img)
    assert np.array_equal(out, _oracle_decode(oracle, ef))


def test_single_symbol_alphabet(mh, device):
    img = np.zeros((64, 128), np.uint8)  # every delta 0 -> one symbol, code "0"
    ef = mh.encode_frame(img)
    assert int((ef.canon > 0).sum()) == 1 and ef.canon.max() == 1
    assert np.array_equal(_decode([ef], device)[0], img)


def test_global_path_long_span(mh, oracle, device):
    """A tile whose code span exceeds the LDS window decodes from global memory."""
    d = long_span_deltas(1024, 256)
    img = image_from_block_deltas(d, 1024, 256)
    ef = mh.encode_frame(img)
    assert (int(ef.block_offsets[64]) - int(ef.block_offsets[0])) // 8 > 4352
    out = _decode([ef], device)[0]
    assert np.array_equal(out, img)
    assert np.array_equal(out, _oracle_decode(oracle, ef))


def test_tile_8192_roundtrip(mh, device, bigbridge):
    """Full-size config 3: decode(encode(x)) == x (size-independent property)."""
    from metalhuffman_amd import frames as F
    img = F.mirror_tile(bigbridge, 8192, 8192)
    ef = mh.encode_frame(img)
    out = _decode([ef], device)[0]
    assert np.array_equal(out, img)


def test_garbage_stream_no_fault(mh, device, bigbridge):
    """Corrupt codes with valid tables/offsets: must complete without a fault."""
    ef = mh.encode_frame(np.ascontiguousarray(bigbridge[:768, :1024]))
    bad = np.random.default_rng(5).integers(0, 256, size=ef.codes.size, dtype=np.uint8)
    bad[-4:] = 0
    ef.codes = bad
    out = _decode([ef], device)[0]
    assert out.shape == (768, 1024)


def test_raster_beyond_2_gib(mh, device):
    """Maximum-size corner: a 65535-wide frame whose raster exceeds 2 GiB (and the
    u32 store range of one descriptor). Encoded and checked on the device only."""
    import torch
    from metalhuffman_amd import decoder as D
    from metalhuffman_amd.encoder import encode_frame_device
    W, H = 65535, 32800
    y = torch.arange(H, device=device, dtype=torch.int32).view(H, 1) // 8
    x = torch.arange(W, device=device, dtype=torch.int32).view(1, W) // 8
    img = ((x * 7 + y * 3) & 0xFF).to(torch.uint8).contiguous()  # one value per 8x8 block
    assert img.numel() > 2 ** 31
    ef = encode_frame_device(img)
    t1, t2 = mh.Huffman.generateSplitLookupTables(ef.canon)
    out = D.decode(ef.frames(), D.DeviceTables.upload(t1, t2, device))
    torch.cuda.synchronize(device)
    assert torch.equal(out[0, :, :W], img)
    del out, ef, img
    torch.cuda.empty_cache()


def test_small_launch_multi_frame(mh, oracle, device, bigbridge):
    """A few frames in one launch (frame code offsets) take the one-tile-per-wave
    kernel: 3 x 192 tiles, 14-bit table."""
    from metalhuffman_amd import frames as F
    base = np.ascontiguousarray(bigbridge[:1024, :768])
    imgs = [F.block_shuffle(base, s) if s else base for s in range(3)]
    efs = [mh.encode_frame(im) for im in imgs]
    assert efs[0].canon.max() <= 14
    out = _decode(efs, device)
    for i, (im, ef) in enumerate(zip(imgs, efs)):
        assert np.array_equal(out[i], im), i
        assert np.array_equal(out[i], _oracle_decode(oracle, ef)), i


@pytest.mark.parametrize("mode", ["long_codes", "no_delta", "init_zero_delta"])
def test_small_launch_multi_frame_variants(mh, oracle, device, bigbridge, mode):
    """Multi-frame small launches with the 13-bit table (16-bit codes), raw symbols,
    and per-block init bytes."""
    from metalhuffman_amd import frames as F
    if mode == "long_codes":
        d = fibonacci_deltas(17, 256 * 256, seed=11)
        base = image_from_block_deltas(d, 256, 256)
        kw = {}
    elif mode == "no_delta":
        base = fibonacci_deltas(17, 256 * 256, seed=12).reshape(256, 256)
        kw = {"flags": mh.MH_FLAG_NO_DELTA}
    else:
        base = np.ascontiguousarray(bigbridge[:768, :1024])
        kw = {"init_zero_delta": True}
    imgs = [F.block_shuffle(base, 40 + s) for s in range(3)]
    efs = [mh.encode_frame(im, **kw) for im in imgs]
    out = _decode(efs, device)
    for i, (im, ef) in enumerate(zip(imgs, efs)):
        assert np.array_equal(out[i], im), i
        assert np.array_equal(out[i], _oracle_decode(oracle, ef)), i


@pytest.mark.parametrize("n_sym", [15, 17])
@pytest.mark.parametrize("delta", [True, False])
def test_small_kernel_refill_extremes(mh, oracle, device, n_sym, delta):
    """The single-frame kernel's lazy refill (refill test on the cursor a lookup used,
    applied one step later) at its deepest cursor: blocks of p = 0..32 one-bit codes and
    then runs of the longest codes (14 bits: the 14-bit table; 16 bits: the 13-bit table
    with escapes), so lookups see every bit alignment up to 47 bits into the window.
    512x512 = 64 tiles, one launch of the small kernel; bit-exact vs input and oracle."""
    d = refill_extreme_deltas(n_sym, 512, 512, seed=n_sym)
    if delta:
        img = image_from_block_deltas(d, 512, 512)
        ef = mh.encode_frame(img)
    else:  # raw symbols: the raster whose block split is d itself
        img = np.ascontiguousarray(d.reshape(64, 64, 8, 8).transpose(0, 2, 1, 3).reshape(512, 512))
        ef = mh.encode_frame(img, flags=mh.MH_FLAG_NO_DELTA)
    assert ef.canon.max() == n_sym - 1
    out = _decode([ef], device)[0]
    assert np.array_equal(out, img)
    assert np.array_equal(out, _oracle_decode(oracle, ef))


@pytest.mark.parametrize("h", [2048, 2056])
def test_small_batch_kernel_boundary(mh, device, bigbridge, h):
    """2048x2048 = 1024 tiles (the small kernel's limit on a 256-CU part) and
    2048x2056 = 1028 tiles (the batch kernel): same bytes either side."""
    from metalhuffman_amd import frames as F
    img = F.mirror_tile(bigbridge, h, 2048)
    ef = mh.encode_frame(img)
    out = _decode([ef], device)[0]
    assert np.array_equal(out, img)


@pytest.mark.parametrize("n_sym", [14, 15])
def test_batch_kernel_code_length_paths(mh, oracle, device, n_sym):
    """20 frames x 64 tiles (> the small kernel's limit): longest code 13 bits takes
    the batch kernel's escape-free step, 14 bits the escape step."""
    from metalhuffman_amd import frames as F
    d = fibonacci_deltas(n_sym, 512 * 512, seed=30 + n_sym)
    base = image_from_block_deltas(d, 512, 512)
    imgs = [F.block_shuffle(base, 200 + s) for s in range(20)]
    efs = [mh.encode_frame(im) for im in imgs]
    assert efs[0].canon.max() == n_sym - 1
    out = _decode(efs, device)
    for i, im in enumerate(imgs):
        assert np.array_equal(out[i], im), i
    assert np.array_equal(out[7], _oracle_decode(oracle, efs[7]))


def test_fuzz_shapes_and_histograms(mh, oracle, device):
    """Seeded fuzz: 40 frames of random size (1..700 each side), random symbol
    histograms (geometric / two-sided / uniform), all three formats, prepared and
    in-kernel tables; every output equals the oracle's shader-semantics decode."""
    r = np.random.default_rng(2024)
    done = 0
    for i in range(60):
        h, w = int(r.integers(1, 701)), int(r.integers(1, 701))
        kind = i % 3
        if kind == 0:
            img = np.minimum(r.geometric(r.uniform(0.05, 0.6), size=(h, w)) - 1, 255).astype(np.uint8)
            img = np.cumsum(img, axis=1, dtype=np.uint8)
        elif kind == 1:
            img = (np.round(r.normal(128, r.uniform(1, 30), size=(h, w))) % 256).astype(np.uint8)
        else:
            img = r.integers(0, 256, size=(h, w), dtype=np.uint8)
        fmt = int(r.integers(0, 3))
        kw = {"flags": mh.MH_FLAG_NO_DELTA} if fmt == 1 else ({"init_zero_delta": True} if fmt == 2 else {})
        try:
            ef = mh.encode_frame(img, **kw)
        except mh.MHError:
            continue  # a code deeper than 16 bits: invalid for the reference too
        out = _decode([ef], device, prepared=bool(i % 2))[0]
        assert np.array_equal(out, img), (i, h, w, kind, fmt)
        assert np.array_equal(out, _oracle_decode(oracle, ef)), (i, h, w, kind, fmt)
        done += 1
        if done == 40:
            break
    assert done >= 30


def test_batch_kernel_flat_table(mh, oracle, device):
    """Uniform random bytes: every code 8 bits (a flat table), every block exactly
    64 bytes -> the batch kernel's swizzled-stage step; 5 x 1024^2 = 1280 tiles."""
    from metalhuffman_amd import frames as F
    base = F.uniform_random(1024, 1024, 77)
    imgs = [base] + [F.block_shuffle(base, 300 + s) for s in range(4)]
    efs = [mh.encode_frame(im) for im in imgs]
    assert efs[0].canon.min() == efs[0].canon.max() == 8
    out = _decode(efs, device)
    for i, im in enumerate(imgs):
        assert np.array_equal(out[i], im), i
    assert np.array_equal(out[3], _oracle_decode(oracle, efs[3]))


def _shift_stream(ef, k: int):
    """The same frame with its code stream moved k bits later (k leading zero bits) and
    every block offset with it: blocks off the byte grid, which no reference producer
    writes but the buffer contract allows."""
    import dataclasses
    from metalhuffman_amd import _native as N
    bits = np.unpackbits(ef.codes[: ef.payload_bytes])
    moved = np.packbits(np.concatenate([np.zeros(k, np.uint8), bits]))
    codes = np.concatenate([moved, np.zeros(N.MH_CODES_PAD, np.uint8)])
    return dataclasses.replace(ef, codes=codes, block_offsets=(ef.block_offsets + np.uint32(k)).astype(np.uint32))


@pytest.mark.parametrize("n", [1, 5])
@pytest.mark.parametrize("fmt", ["delta", "no_delta", "block_init", "edges", "flat4", "off_grid"])
def test_flat8_paths(mh, oracle, device, fmt, n):
    """Flat 8-bit tables (uniform bytes: every code 8 bits, code c = symbol c) decode with
    byte arithmetic instead of the lookup chain: n = 1 frame (256 tiles, the single-frame
    kernel, from its staged span) and n = 5 frames (1,280+ tiles, the batch kernel, per-lane
    code loads). Formats: delta, raw symbols, per-block init bytes (attached to flat frames:
    the reference's init-byte producer always makes symbol 0 shorter), partial edge
    blocks and rows past H (1032x1008 frames decoded as 1027x1001: the same block grid),
    a flat 4-bit table (16 symbols: the general flat step), and blocks off the byte grid
    (the general flat step, from the slow loop)."""
    import dataclasses
    from metalhuffman_amd import frames as F
    kw = {}
    if fmt == "edges":
        base = F.uniform_random(1008, 1032, 5)
    elif fmt == "flat4":
        base = (F.uniform_random(1024, 1024, 6) & 15).astype(np.uint8)
        kw = {"flags": mh.MH_FLAG_NO_DELTA}
    else:
        base = F.uniform_random(1024, 1024, 7)
    if fmt == "no_delta":
        kw = {"flags": mh.MH_FLAG_NO_DELTA}
    imgs = [base] + [F.block_shuffle(base, 700 + s) for s in range(1, n)]
    efs = [mh.encode_frame(im, **kw) for im in imgs]
    L = efs[0].canon[efs[0].canon > 0]
    assert L.min() == L.max() == (4 if fmt == "flat4" else 8), (L.min(), L.max())
    if fmt == "off_grid":
        efs = [_shift_stream(ef, 3 + i) for i, ef in enumerate(efs)]
    elif fmt == "block_init":
        r = np.random.default_rng(8)
        efs = [dataclasses.replace(ef, block_init=r.integers(0, 256, ef.n_blocks, dtype=np.uint8)) for ef in efs]
    elif fmt == "edges":
        efs = [dataclasses.replace(ef, width=1027, height=1001) for ef in efs]
        imgs = [im[:1001, :1027] for im in imgs]
    out = _decode(efs, device)
    for i, (im, ef) in enumerate(zip(imgs, efs)):
        if fmt != "block_init":
            assert np.array_equal(out[i], im), i
        assert np.array_equal(out[i], _oracle_decode(oracle, ef)), i


MAXLEN_OFF = 18464 + 32768  # mh_lut.hpp kMaxLenOff: [longest, shortest, flat8, 0] (u32)


def _lens_word(tabs):
    return tabs.lut[MAXLEN_OFF: MAXLEN_OFF + 16].cpu().numpy().view(np.uint32).tolist()


def test_flat8_flag_follows_every_first_level_entry(mh, oracle, device):
    """the byte-arithmetic path is taken only for the identity 8-bit code (code c =
    symbol c at EVERY first-level entry). Since round 6 the table builders decide it once and
    record it in the prepared table's flat8 word (mh_lut.hpp), which both kernels read:
    mh_prepare_lut from every first-level entry, mh_build_tables_device from the canonical
    lengths (all 256 symbols at 8 bits). A flat 8-bit table with two symbols' codes swapped --
    legal T1/T2 for mh_prepare_lut, every code still 8 bits -- must get flat8 = 0 and decode
    through the lookup chain exactly as the oracle decodes it, in the single-frame kernel (one
    frame) and the batch kernel (5 frames); 255 symbols at 8 bits (an incomplete code) gets 0
    from both builders."""
    import torch
    from metalhuffman_amd import decoder as D
    from metalhuffman_amd import frames as F
    imgs = [F.uniform_random(1024, 1024, 11)] + [F.block_shuffle(F.uniform_random(1024, 1024, 11), 900 + s)
                                                 for s in range(4)]
    efs = [mh.encode_frame(im) for im in imgs]
    t1, t2 = efs[0].tables()
    assert _lens_word(D.DeviceTables.upload(t1, t2, device)) == [8, 8, 1, 0]
    assert _lens_word(D.DeviceTables.from_canonical_header(efs[0].canon, device)) == [8, 8, 1, 0]
    t1p = t1.copy()
    t1p[2 * 0x5A], t1p[2 * 0x5B] = t1[2 * 0x5B], t1[2 * 0x5A]   # {symbol, width}: swap two symbols
    tabs = D.DeviceTables.upload(t1p, t2, device)
    assert _lens_word(tabs) == [8, 8, 0, 0]
    for fl in (efs[:1], efs):
        fr = D.DeviceFrames.pack(fl, device)
        out = D.decode(fr, tabs)
        torch.cuda.synchronize(device)
        for i, ef in enumerate(fl):
            want = oracle.decode_frame_shader(ef.block_offsets, ef.codes, t1p, t2, ef.width, ef.height,
                                              block_init=ef.block_init, delta=True)
            got = out[i, :, : fr.width].cpu().numpy()
            assert not np.array_equal(got, imgs[i]) and np.array_equal(got, want), (len(fl), i)
    canon = np.full(256, 8, np.uint8)
    canon[77] = 0
    dev = D.DeviceTables.from_canonical_header(canon, device)
    host_t1, host_t2 = mh.codec.Huffman.generateSplitLookupTables(canon)
    assert _lens_word(dev)[2] == 0
    assert _lens_word(D.DeviceTables.upload(host_t1, host_t2, device))[2] == 0


def test_both_kernels_follow_the_flat8_word(mh, device):
    """ADVICE r05's concern -- the two kernels decoding one frame differently from one prepared
    table -- cannot arise since round 6: both act on the same flat8 word. A prepared table whose
    entries were changed after the builder set the word (outside the contract: the buffer is
    opaque, metalhuffman.h) decodes the same way in the single-frame kernel (one frame) and
    the batch kernel (5 frames): by the word, i.e. the byte path, here the image."""
    import torch
    from metalhuffman_amd import decoder as D
    from metalhuffman_amd import frames as F
    imgs = [F.uniform_random(1024, 1024, 12)] + [F.block_shuffle(F.uniform_random(1024, 1024, 12), 700 + s)
                                                 for s in range(4)]
    efs = [mh.encode_frame(im) for im in imgs]
    t1, t2 = efs[0].tables()
    tabs = D.DeviceTables.upload(t1, t2, device)
    assert _lens_word(tabs) == [8, 8, 1, 0]
    lut16 = tabs.lut.view(torch.int16)
    c, wrong = 0x5A, (((0x5A ^ 1) << 8) - 8) & 0xFFFF
    w = torch.tensor([wrong], dtype=torch.int32, device=device).to(torch.int16)
    lut16[(c << 5) | 1] = w[0]                       # 13-bit first level
    lut16[18464 // 2 + ((c << 6) | 2)] = w[0]         # 14-bit table
    outs = []
    for fl in (efs[:1], efs):
        fr = D.DeviceFrames.pack(fl, device)
        out = D.decode(fr, tabs)
        torch.cuda.synchronize(device)
        outs.append(out[0, :, : fr.width].cpu().numpy())
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], imgs[0])


@pytest.mark.parametrize("kind", ["flat", "flat4", "noesc", "general"])
def test_batch_kernel_multi_tile_waves_per_flavour(mh, device, bigbridge, kind):
    """Every step flavour of the batch kernel (one persistent-loop instantiation each)
    through its pipelined multi-tile loop: more tiles than resident waves (256 CUs x 24
    waves), so waves decode 2+ tiles with the next span in flight. flat: uniform random
    bytes (every code 8 bits, swizzled stage); noesc: the 8192-wide mirror tile (longest
    code 13 bits); general: BigBridge shuffles (14-bit codes, escape test). The round-5
    bisect found a flat-flavour failure here that no 1-tile-per-wave test could see."""
    import torch
    from metalhuffman_amd import decoder as D
    from metalhuffman_amd import frames as F
    if kind == "flat":  # since round 5 the flat 8-bit byte-arithmetic loop (flat8_loop)
        base = F.uniform_random(1024, 1024, 91)
    elif kind == "flat4":  # a flat 4-bit table: the swizzled-stage lookup loop (Lut13Flat), the one
        base = (F.uniform_random(1024, 1024, 92) & 15).astype(np.uint8)  # round 5's spilled build broke
    elif kind == "noesc":
        base = F.mirror_tile(bigbridge, 2048, 8192)
    else:
        base = np.ascontiguousarray(bigbridge[:1024, :1024])
    n = max(1, -(-8400 * 64 // (base.size // 64)))  # > 8,192 tiles of 64 blocks
    imgs = [base] + [F.block_shuffle(base, 500 + s) for s in range(n - 1)]
    efs = [mh.encode_frame(im, **({"flags": mh.MH_FLAG_NO_DELTA} if kind == "flat4" else {})) for im in imgs]
    mx, mn = int(efs[0].canon.max()), int(efs[0].canon[efs[0].canon > 0].min())
    assert {"flat": mx == mn == 8, "flat4": mx == mn == 4, "noesc": mx <= 13, "general": mx > 13}[kind], mx
    t1, t2 = efs[0].tables()
    tabs = D.DeviceTables.upload(t1, t2, device)
    fr = D.DeviceFrames.pack(efs, device)
    out = D.decode(fr, tabs)
    torch.cuda.synchronize(device)
    ref = torch.from_numpy(np.stack(imgs)).to(device)
    bad = [i for i in range(n) if not torch.equal(out[i, :, : fr.width], ref[i])]
    assert not bad, (kind, bad[:8])


@pytest.mark.parametrize("prepared", [True, False])
@pytest.mark.parametrize("flags", [0, 1])
def test_zero_width_windows_match_reference(mh, oracle, device, prepared, flags):
    """Windows the table does not decode ({0,0}: the reference's dummy T2 subtable,
    HuffmanUtil.cpp:550-556) consume nothing and yield symbol 0 -- prev repeats with
    deltas, the byte is 0 without (AAPLShaders.metal:241-268). A single-symbol
    alphabet has the one code '0', so all-ones code bytes hit that entry on every
    lookup; both kernels (prepared table: small-launch; in-kernel table: batch)."""
    from metalhuffman_amd import codec as C
    img = np.zeros((24, 40), np.uint8)
    ef = mh.encode_frame(img, flags=flags)
    bad = C.EncodedFrame(ef.width, ef.height, ef.canon, np.full_like(ef.codes, 0xFF),
                         ef.block_offsets, None, ef.flags)
    out = _decode([bad, bad], device, prepared)
    ref = _oracle_decode(oracle, bad)
    assert not ref.any()
    assert np.array_equal(out[0], ref) and np.array_equal(out[1], ref)


@pytest.mark.parametrize("world", [2, 3, 7])
def test_single_frame_bands(mh, device, bigbridge, world):
    """Single-frame split: each band, rebased to its own code
    bytes, decodes on the GPU to exactly its rows of the frame (full BigBridge, a
    partial-block crop with init bytes)."""
    from metalhuffman_amd import dist as MD
    for img, kw in ((bigbridge, {}), (np.ascontiguousarray(bigbridge[:777, :1001]), {"init_zero_delta": True})):
        ef = mh.encode_frame(img, **kw)
        rows = []
        for r in range(world):
            band, y0 = MD.frame_band(ef, world, r)
            out = _decode([band], device)[0]
            assert np.array_equal(out, img[y0: y0 + band.height]), (img.shape, world, r)
            rows.append(out)
        assert np.array_equal(np.concatenate(rows), img)


def test_config4_full_shard_one_launch(mh, oracle, device, bigbridge):
    """BASELINE config 4 at its per-GPU size: a 64-frame block-shuffled shard (512
    frames / 8 GPUs) decoded in ONE launch of the batch kernel. Every frame equals its
    input; two frames also equal the oracle's shader-semantics decode (the DEBUG
    self-check of Shared/AAPLRenderer.m:616-650, here against the restatement)."""
    import torch
    from metalhuffman_amd import decoder as D
    from metalhuffman_amd import frames as F
    imgs = [F.block_shuffle(bigbridge, 5000 + s) for s in range(64)]
    import concurrent.futures as cf
    with cf.ThreadPoolExecutor(8) as ex:  # ctypes releases the GIL
        efs = list(ex.map(mh.encode_frame, imgs))
    t1, t2 = efs[0].tables()
    tabs = D.DeviceTables.upload(t1, t2, device)
    fr = D.DeviceFrames.pack(efs, device)
    assert fr.n_frames == 64
    out = D.decode(fr, tabs)
    ref = torch.from_numpy(np.stack(imgs)).to(device)
    torch.cuda.synchronize(device)
    bad = [i for i in range(64) if not torch.equal(out[i, :, :2048], ref[i])]
    assert not bad, bad
    for i in (0, 41):
        assert np.array_equal(out[i, :, :2048].cpu().numpy(), _oracle_decode(oracle, efs[i])), i


@pytest.mark.parametrize("lane_pairs", [False, True])
def test_any_order_run_of_frames(mh, oracle, device, bigbridge, lane_pairs):
    """MH_FLAG_ANY_ORDER: a run of one-frame launches on one stream, every launch after
    the first without the dispatch barrier (it may start while the previous decode
    drains), each into its own raster -- the bench's timed region. Then a launch WITHOUT
    the flag reuses frame 0's raster for another frame: stream order still holds for it.
    Every raster equals its input; frame 3 also equals the oracle's decode."""
    import torch
    from metalhuffman_amd import _native as N
    from metalhuffman_amd import decoder as D
    from metalhuffman_amd import frames as F
    imgs = [F.block_shuffle(bigbridge, 7000 + s) for s in range(12)]
    efs = [mh.encode_frame(im) for im in imgs]
    t1, t2 = efs[0].tables()
    tabs = D.DeviceTables.upload(t1, t2, device)
    frs = [D.DeviceFrames.pack([ef], device) for ef in efs]
    outs = [torch.full((1, 1536, 2048), 0xA5, dtype=torch.uint8, device=device) for _ in efs]
    extra = N.MH_FLAG_LANE_PAIRS if lane_pairs else 0
    for rep in range(3):
        for i, fr in enumerate(frs[:-1]):
            D.decode(fr, tabs, outs[i], extra_flags=extra | (N.MH_FLAG_ANY_ORDER if i else 0))
    D.decode(frs[-1], tabs, outs[0], extra_flags=extra)  # barrier launch: after every earlier one
    torch.cuda.synchronize(device)
    ref = torch.from_numpy(np.stack(imgs)).to(device)
    assert torch.equal(outs[0][0], ref[-1])
    bad = [i for i in range(1, len(efs) - 1) if not torch.equal(outs[i][0], ref[i])]
    assert not bad, bad
    assert np.array_equal(outs[3][0].cpu().numpy(), _oracle_decode(oracle, efs[3]))


def test_cached_frame_struct_follows_buffers(mh, device, bigbridge):
    """decoder.decode keeps the mh_frame struct on the DeviceFrames (the per-call Python
    cost is what an eager caller pays per frame): swapping a buffer tensor, the tables or
    the extra flags must give a fresh struct, and a too-small / wrong-device `out` is refused
    before anything launches."""
    import torch
    from metalhuffman_amd import _native as N, decoder as D, frames as F
    a = mh.encode_frame(bigbridge)
    b = mh.encode_frame(F.block_shuffle(bigbridge, 3))
    t1, t2 = a.tables()
    tabs = D.DeviceTables.upload(t1, t2, device)
    fa, fb = D.DeviceFrames.pack([a], device), D.DeviceFrames.pack([b], device)
    out = D.decode(fa, tabs)
    assert np.array_equal(out[0, :, :2048].cpu().numpy(), bigbridge)
    s0 = D._frame_struct(fa, tabs)
    assert D._frame_struct(fa, tabs) is s0  # reused while nothing changed
    assert D._frame_struct(fa, tabs, N.MH_FLAG_ANY_ORDER).flags == s0.flags | N.MH_FLAG_ANY_ORDER
    # re-seat frame a's buffers with frame b's: the cache must follow
    fa.codes, fa.block_offsets = fb.codes, fb.block_offsets
    D.decode(fa, tabs, out, extra_flags=N.MH_FLAG_ANY_ORDER)
    torch.cuda.synchronize(device)
    assert np.array_equal(out[0, :, :2048].cpu().numpy(), F.block_shuffle(bigbridge, 3))
    assert D._frame_struct(fa, tabs).d_codes == fb.codes.data_ptr()
    # new tables object (same contents): new struct pointing at its buffers
    tabs2 = D.DeviceTables.upload(t1, t2, device)
    assert D._frame_struct(fa, tabs2).d_lut == tabs2.lut.data_ptr()
    with pytest.raises(ValueError):
        D.decode(D.DeviceFrames.pack([a, b], device), tabs, out)  # room for 1 frame, not 2
    with pytest.raises(ValueError):
        D.decode(fa, tabs, torch.empty_like(out, device="cpu"))
