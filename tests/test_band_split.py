"""Single-frame split: a band of block rows, rebased to its own
code bytes, decodes (oracle, shader semantics) to exactly those rows of the frame."""
from __future__ import annotations

import numpy as np
import pytest

from helpers import fibonacci_deltas


def _frames():
    from metalhuffman_amd import frames as F
    bb = F.bigbridge()
    yield "bigbridge_768x1024", np.ascontiguousarray(bb[:768, :1024]), {}
    yield "crop_777x1001", np.ascontiguousarray(bb[:777, :1001]), {}
    yield "init_zero", np.ascontiguousarray(bb[:257, :333]), {"init_zero_delta": True}
    yield "no_delta", fibonacci_deltas(15, 200 * 136, seed=2).reshape(200, 136), {"flags": 1}


@pytest.mark.parametrize("world", [1, 2, 3, 5])
def test_bands_decode_to_frame_rows(world):
    import metalhuffman_amd as mh
    from metalhuffman_amd import dist as MD
    from oracle import oracle as O
    for name, img, kw in _frames():
        ef = mh.encode_frame(img, **kw)
        t1, t2 = ef.tables()
        rows = []
        for r in range(world):
            band, y0 = MD.frame_band(ef, world, r)
            if band is None:
                continue
            assert y0 == sum(x.shape[0] for x in rows)
            assert band.codes.size <= ef.codes.size
            out = O.decode_frame_shader(band.block_offsets, band.codes, t1, t2, band.width, band.height,
                                        band.block_init, delta=not (ef.flags & 1))
            assert np.array_equal(out, img[y0: y0 + band.height]), (name, world, r)
            rows.append(out)
        assert np.array_equal(np.concatenate(rows), img), name


def test_band_bounds():
    import metalhuffman_amd as mh
    from metalhuffman_amd import frames as F
    ef = mh.encode_frame(np.ascontiguousarray(F.bigbridge()[:64, :64]))
    with pytest.raises(ValueError):
        ef.band(3, 3)
    with pytest.raises(ValueError):
        ef.band(0, 9)
    b = ef.band(7, 8)           # last block row
    assert b.height == 8 and b.block_offsets[0] == ef.block_offsets[56] % 8


def test_more_ranks_than_block_rows():
    import metalhuffman_amd as mh
    from metalhuffman_amd import dist as MD
    from metalhuffman_amd import frames as F
    from oracle import oracle as O
    img = np.ascontiguousarray(F.bigbridge()[:20, :40])   # 3 block rows
    ef = mh.encode_frame(img)
    t1, t2 = ef.tables()
    got = []
    for r in range(5):
        band, y0 = MD.frame_band(ef, 5, r)
        if band is None:
            continue
        got.append(O.decode_frame_shader(band.block_offsets, band.codes, t1, t2, band.width, band.height))
    assert len(got) == 3 and np.array_equal(np.concatenate(got), img)
