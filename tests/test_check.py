"""The decode contract's debug mode ("Errors"): mh_check reports
zero-width lookups, escapes past T2 and blocks whose codes miss the next block's
offset, without touching a raster. CPU tests pin the oracle's report on streams
with known defects; GPU tests require the product's report to equal the oracle's."""
from __future__ import annotations

import numpy as np
import pytest

from helpers import fibonacci_deltas, image_from_block_deltas

CLEAN = [0, 0, 0, 0xFFFFFFFF]


def _frame(mh, img, **kw):
    return mh.encode_frame(img, **kw)


def _single_symbol_frame(mh):
    """All-zero image: one symbol, code '0' -- an incomplete code, so any '1' bit
    in a window is a lookup no code matches."""
    ef = mh.encode_frame(np.zeros((16, 32), np.uint8))
    assert int((ef.canon > 0).sum()) == 1
    return ef


def test_oracle_clean_streams(mh, oracle, bigbridge):
    for img in (bigbridge, np.ascontiguousarray(bigbridge[:777, :1001])):
        ef = _frame(mh, img)
        t1, t2 = ef.tables()
        assert oracle.check_frame(ef.block_offsets, ef.codes, t1, t2).tolist() == CLEAN
    d = fibonacci_deltas(17, 256 * 256, seed=5)  # 16-bit codes through T2
    ef = _frame(mh, image_from_block_deltas(d, 256, 256))
    t1, t2 = ef.tables()
    assert oracle.check_frame(ef.block_offsets, ef.codes, t1, t2).tolist() == CLEAN


def test_oracle_offset_mismatch(mh, oracle, bigbridge):
    ef = _frame(mh, np.ascontiguousarray(bigbridge[:256, :256]))
    t1, t2 = ef.tables()
    offs = ef.block_offsets.copy()
    offs[5] += 1  # block 4's codes now end one bit before block 5's recorded start
    rep = oracle.check_frame(offs, ef.codes, t1, t2)
    assert rep[2] >= 1 and rep[3] == 4


def test_oracle_zero_width(mh, oracle):
    ef = _single_symbol_frame(mh)
    t1, t2 = ef.tables()
    codes = ef.codes.copy()
    codes[0] = 0x80  # block 0's first window starts with a '1'
    rep = oracle.check_frame(ef.block_offsets, codes, t1, t2)
    # the lookup never advances: every one of block 0's 64 steps is zero width,
    # and block 0 ends where it started (offset 0 != offset of block 1 = 64)
    assert rep[0] == 64 and rep[1] == 0 and rep[2] == 1 and rep[3] == 0


def test_oracle_escape_past_t2(mh, oracle, bigbridge):
    ef = _frame(mh, bigbridge)
    t1, t2 = ef.tables()
    rep = oracle.check_frame(ef.block_offsets, ef.codes, t1, t2[:512])  # only 1 real subtable
    assert rep[1] > 0 and rep[3] != 0xFFFFFFFF


# ---------------------------------------------------------------------------- GPU
def _gpu_check(efs, device, t1=None, t2=None, codes=None, offsets=None):
    from metalhuffman_amd import decoder as D
    if t1 is None:
        t1, t2 = efs[0].tables()
    if codes is not None or offsets is not None:
        import dataclasses
        efs = [dataclasses.replace(efs[0], codes=codes if codes is not None else efs[0].codes,
                                   block_offsets=offsets if offsets is not None else efs[0].block_offsets)]
    tabs = D.DeviceTables.upload(t1, t2, device)
    fr = D.DeviceFrames.pack(efs, device)
    return D.check(fr, tabs).cpu().numpy()


@pytest.mark.gpu
def test_gpu_check_clean_and_batch(mh, oracle, device, bigbridge):
    from metalhuffman_amd import frames as F
    efs = [mh.encode_frame(F.block_shuffle(bigbridge, s)) for s in range(3)]
    rep = _gpu_check(efs, device)
    assert rep.tolist() == [CLEAN] * 3


@pytest.mark.gpu
def test_gpu_check_matches_oracle_on_defects(mh, oracle, device, bigbridge):
    # offset mismatch
    ef = mh.encode_frame(np.ascontiguousarray(bigbridge[:256, :256]))
    t1, t2 = ef.tables()
    offs = ef.block_offsets.copy()
    offs[5] += 1
    got = _gpu_check([ef], device, offsets=offs)[0]
    assert got.tolist() == oracle.check_frame(offs, ef.codes, t1, t2).tolist()
    # zero-width lookups (incomplete single-symbol code)
    ef = _single_symbol_frame(mh)
    t1, t2 = ef.tables()
    codes = ef.codes.copy()
    codes[0] = 0x80
    got = _gpu_check([ef], device, codes=codes)[0]
    assert got.tolist() == oracle.check_frame(ef.block_offsets, codes, t1, t2).tolist()
    # escapes past a truncated T2, and a garbage bitstream
    ef = mh.encode_frame(bigbridge)
    t1, t2 = ef.tables()
    got = _gpu_check([ef], device, t1=t1, t2=t2[:512])[0]
    assert got.tolist() == oracle.check_frame(ef.block_offsets, ef.codes, t1, t2[:512]).tolist()
    bad = np.random.default_rng(9).integers(0, 256, size=ef.codes.size, dtype=np.uint8)
    got = _gpu_check([ef], device, codes=bad)[0]
    want = oracle.check_frame(ef.block_offsets, bad, t1, t2)
    assert got.tolist() == want.tolist() and want[2] > 0
