"""GPU parity of the experimental lane-pair single-frame kernel (MH_FLAG_LANE_PAIRS).

north_star's lane-group cursor: each 8x8 block is decoded by two lanes, one from
the block's first bit and one speculatively from its middle bit, re-synchronised
through ds_bpermute. Whatever the meeting point -- or none --
the bytes must equal the oracle's restatement of AAPLShaders.metal:127-365 and the
default kernel's. Bit-exact, like every decode test.
"""
from __future__ import annotations

import numpy as np
import pytest

from helpers import fibonacci_deltas, image_from_block_deltas, lane_pair_oversize_deltas

pytestmark = pytest.mark.gpu


def _decode(efs, device, lane_pairs=True, prepared=True):
    import torch
    import metalhuffman_amd as mh
    from metalhuffman_amd import decoder as D
    t1, t2 = efs[0].tables()
    tabs = D.DeviceTables.upload(t1, t2, device, prepare_lut=prepared)
    fr = D.DeviceFrames.pack(efs, device)
    out = D.decode(fr, tabs, extra_flags=mh.MH_FLAG_LANE_PAIRS if lane_pairs else 0)
    torch.cuda.synchronize(device)
    return out[..., : fr.width].cpu().numpy()


def _oracle(O, ef):
    t1, t2 = ef.tables()
    return O.decode_frame_shader(ef.block_offsets, ef.codes, t1, t2, ef.width, ef.height,
                                 block_init=ef.block_init, delta=not (ef.flags & 1))


def test_bigbridge_config2(mh, oracle, device, bigbridge):
    """The headline frame (2048x1536, 14-bit table)."""
    ef = mh.encode_frame(bigbridge)
    out = _decode([ef], device)[0]
    assert np.array_equal(out, bigbridge)
    assert np.array_equal(out, _oracle(oracle, ef))


def test_block_shuffled_frames(mh, device, bigbridge):
    """Several config-4 frames in one small launch (frame code offsets)."""
    from metalhuffman_amd import frames as F
    base = np.ascontiguousarray(bigbridge[:1024, :768])
    imgs = [F.block_shuffle(base, s) for s in range(3)]
    efs = [mh.encode_frame(im) for im in imgs]
    out = _decode(efs, device)
    for i, im in enumerate(imgs):
        assert np.array_equal(out[i], im), i


@pytest.mark.parametrize("hw", [(1, 1), (7, 9), (9, 7), (1001, 777), (5, 2051), (64, 520)])
def test_odd_sizes(mh, oracle, device, bigbridge, hw):
    """Partial blocks, one-block frames, a 32-block tile spanning two block rows."""
    h, w = hw
    img = np.ascontiguousarray(np.tile(bigbridge, (1 + h // 1536, 1 + w // 2048))[:h, :w])
    ef = mh.encode_frame(img)
    out = _decode([ef], device)[0]
    assert np.array_equal(out, img)
    assert np.array_equal(out, _oracle(oracle, ef))


@pytest.mark.parametrize("n_sym", [15, 17])
def test_long_codes_escape_table(mh, oracle, device, n_sym):
    """Codes of 15-16 bits: the 13-bit table with escapes inside the pair loop."""
    d = fibonacci_deltas(n_sym, 512 * 512, seed=n_sym)
    img = image_from_block_deltas(d, 512, 512)
    ef = mh.encode_frame(img)
    out = _decode([ef], device)[0]
    assert np.array_equal(out, img)
    assert np.array_equal(out, _oracle(oracle, ef))


def test_largest_lane_pair_span(mh, oracle, device):
    """A 32-block tile of 15-bit codes (3,735 B of code bytes) fits the lane-pair stage."""
    img = image_from_block_deltas(lane_pair_oversize_deltas(), 512, 512)
    ef = mh.encode_frame(img)
    o = ef.block_offsets.astype(np.int64)
    assert ef.canon.max() == 15 and (o[32] - o[0]) / 8 > 3712
    out = _decode([ef], device)[0]
    assert np.array_equal(out, img)
    assert np.array_equal(out, _oracle(oracle, ef))


def test_no_delta_and_init_byte(mh, oracle, device, bigbridge):
    """Raw symbols (no running sum to rebase) and per-block init bytes."""
    img = fibonacci_deltas(13, 256 * 256, seed=3).reshape(256, 256)
    ef = mh.encode_frame(img, flags=mh.MH_FLAG_NO_DELTA)
    out = _decode([ef], device)[0]
    assert np.array_equal(out, img) and np.array_equal(out, _oracle(oracle, ef))
    img2 = np.ascontiguousarray(bigbridge[:768, :1024])
    ef2 = mh.encode_frame(img2, init_zero_delta=True)
    out2 = _decode([ef2], device)[0]
    assert np.array_equal(out2, img2) and np.array_equal(out2, _oracle(oracle, ef2))


def test_uniform_and_single_symbol(mh, device):
    """Flat 8-bit codes (every block 512 bits) and the one-symbol alphabet (code '0',
    64-bit blocks: below the speculation threshold, lane A alone)."""
    from metalhuffman_amd import frames as F
    img = F.uniform_random(1024, 512, 9)
    assert np.array_equal(_decode([mh.encode_frame(img)], device)[0], img)
    z = np.zeros((64, 128), np.uint8)
    assert np.array_equal(_decode([mh.encode_frame(z)], device)[0], z)


def test_fuzz_matches_default_kernel(mh, oracle, device):
    """Seeded fuzz over sizes and histograms: lane pairs == default kernel == oracle."""
    r = np.random.default_rng(77)
    done = 0
    for i in range(40):
        h, w = int(r.integers(1, 600)), int(r.integers(1, 600))
        if i % 2:
            img = np.minimum(r.geometric(r.uniform(0.05, 0.6), size=(h, w)) - 1, 255).astype(np.uint8)
            img = np.cumsum(img, axis=1, dtype=np.uint8)
        else:
            img = (np.round(r.normal(128, r.uniform(1, 30), size=(h, w))) % 256).astype(np.uint8)
        try:
            ef = mh.encode_frame(img)
        except mh.MHError:
            continue
        a = _decode([ef], device)[0]
        assert np.array_equal(a, img), (i, h, w)
        assert np.array_equal(a, _decode([ef], device, lane_pairs=False)[0]), (i, h, w)
        done += 1
    assert done >= 25


def test_zero_width_windows_and_garbage(mh, oracle, device, bigbridge):
    """Windows no code matches consume nothing (the reference's {0,0} entry): the
    speculative lane never reaches the block end, so lane A finishes; random code
    bytes must complete without a fault and match the default kernel."""
    from metalhuffman_amd import codec as C
    ef = mh.encode_frame(np.zeros((24, 40), np.uint8))
    bad = C.EncodedFrame(ef.width, ef.height, ef.canon, np.full_like(ef.codes, 0xFF),
                         ef.block_offsets, None, ef.flags)
    assert np.array_equal(_decode([bad], device)[0], _oracle(oracle, bad))
    ef2 = mh.encode_frame(np.ascontiguousarray(bigbridge[:768, :1024]))
    junk = np.random.default_rng(5).integers(0, 256, size=ef2.codes.size, dtype=np.uint8)
    junk[-4:] = 0
    ef2.codes = junk
    # (a garbage frame's last block reads past the payload: the default kernel's
    # behaviour there is the reference for this variant, test_gpu_decode.py only
    # asks it not to fault)
    a = _decode([ef2], device)[0]
    assert np.array_equal(a, _decode([ef2], device, lane_pairs=False)[0])
