"""The product's host codec (libmetalhuffman_amd.so, csrc/mh_host.cpp) is
byte-identical to the oracle on every input: canonical header, codes, block
offsets, T1/T2 and the single 64K table. CPU only."""
from __future__ import annotations

import numpy as np
import pytest

from helpers import fibonacci_deltas, image_from_block_deltas


def _inputs(bigbridge):
    from metalhuffman_amd import frames as F
    r = np.random.default_rng(7)
    yield "bigbridge", bigbridge
    yield "crop", F.crop(bigbridge, 1001, 777)
    yield "random", F.uniform_random(256, 384, 3)
    yield "const0", np.zeros((40, 24), np.uint8)
    yield "const7", np.full((16, 16), 7, np.uint8)
    yield "tiny", np.array([[5]], np.uint8)
    yield "fib17", image_from_block_deltas(fibonacci_deltas(17, 128 * 128, seed=4), 128, 128)
    for i in range(6):
        h, w = int(r.integers(1, 90)), int(r.integers(1, 90))
        yield f"rand{i}", (r.integers(0, 4, size=(h, w)) * r.integers(0, 60)).astype(np.uint8)


def test_encode_frame_identical(mh, oracle, bigbridge):
    for name, img in _inputs(bigbridge):
        ef = mh.encode_frame(img)
        canon, huff, offs = oracle.encode_frame(img)
        assert np.array_equal(ef.canon, canon), name
        assert np.array_equal(ef.codes, huff), name
        assert np.array_equal(ef.block_offsets, offs), name


def test_tables_identical(mh, oracle, bigbridge):
    from metalhuffman_amd.codec import Huffman
    for name, img in _inputs(bigbridge):
        canon, _, _ = oracle.encode_frame(img)
        t1, t2 = Huffman.generateSplitLookupTables(canon)
        o1, o2 = oracle.split_tables(canon)
        assert np.array_equal(t1, o1) and np.array_equal(t2, o2), name
        assert np.array_equal(Huffman.generateLookupTable(canon), oracle.single_table(canon)), name
        assert np.array_equal(Huffman.parseCanonicalHeader(canon), oracle.canonical_codes(canon)), name


def test_encode_huffman_facade(mh, oracle):
    from metalhuffman_amd.codec import Huffman
    r = np.random.default_rng(3)
    for trial in range(20):
        n = 64 * int(r.integers(1, 40))
        sym = r.integers(0, int(r.integers(1, 256)), size=n).astype(np.uint8)
        hdr, canon, codes, offs = Huffman.encodeHuffman(sym, 0, 0, 8)
        c2, k2, o2 = oracle.huffman_encode(sym, 64)
        assert hdr.size == 0  # HuffmanUtil.cpp:1073-1086 drops the file header
        assert np.array_equal(canon, c2) and np.array_equal(codes, k2) and np.array_equal(offs, o2)


def test_signed_byte_deltas(mh, oracle):
    from metalhuffman_amd.codec import Huffman
    r = np.random.default_rng(1)
    a = r.integers(0, 256, size=1000).astype(np.uint8)
    d = Huffman.encodeSignedByteDeltas(a)
    assert np.array_equal(d, oracle.delta_encode(a))
    assert np.array_equal(Huffman.decodeSignedByteDeltas(d), a)


def test_split_merge_blocks(mh, oracle, bigbridge):
    from metalhuffman_amd import codec as C
    for h, w in [(1, 1), (7, 13), (1001, 777), (64, 64)]:
        img = np.ascontiguousarray(bigbridge[:h, :w])
        b = C.split_blocks(img)
        assert np.array_equal(b, oracle.split_blocks(img))
        assert np.array_equal(C.merge_blocks(b, w, h), img)


def test_init_zero_delta_encoding(mh, bigbridge):
    img = np.ascontiguousarray(bigbridge[:256, :256])
    ef = mh.encode_frame(img, init_zero_delta=True)
    from metalhuffman_amd import codec as C
    blocks = C.split_blocks(img)
    assert np.array_equal(ef.block_init, blocks[::64])  # first delta == first pixel


def test_errors(mh):
    from metalhuffman_amd import MHError
    from metalhuffman_amd.codec import Huffman
    img = image_from_block_deltas(fibonacci_deltas(18, 64 * 64 * 4, seed=1), 128, 128)
    with pytest.raises(MHError) as e:
        mh.encode_frame(img)
    assert e.value.status == -3   # MH_ERR_CODE_TOO_LONG (reference: assert codei < 16)
    with pytest.raises(MHError):
        Huffman.encodeHuffman(np.zeros(0, np.uint8), 0, 0, 8)
    with pytest.raises(ValueError):
        Huffman.generateSplitLookupTables(np.zeros(256, np.uint8), 9, 7)
    with pytest.raises(MHError) as e:
        mh.encode_frame(np.zeros((1, 70000), np.uint8))
    assert e.value.status == -2   # MH_ERR_DIMS: beyond the u16 dims uniform


def test_container_header_matches_reference_encoder(mh):
    """HuffmanEncoder::encode's 8-byte header (golden.json, emitted by the real
    reference encoder for every hand-written frame)."""
    from helpers import golden
    for name, fx in golden()["small_frames"].items():
        n = -(-fx["width"] // 8) * -(-fx["height"] // 8) * 64      # symbols after the 8x8 split
        hdr = mh.Huffman.containerHeader(n)
        assert hdr.tobytes().hex() == fx["container_header_hex"], name
        assert mh.Huffman.parseContainerHeader(hdr) == n
    with pytest.raises(mh.MHError):
        mh.Huffman.parseContainerHeader(bytes(8))


def test_flat8_table_is_identity(mh, oracle):
    """The premise of the decoders' flat 8-bit path (mh_decode.hip flat8_*): when every
    code is 8 bits (all 256 symbols, e.g. uniform bytes), canonical assignment gives
    symbol c the code c, so T1 entry c is (symbol c, 8 bits) -- in the product's tables and
    in the oracle's restatement of HuffmanUtil.cpp's split tables alike."""
    from metalhuffman_amd import frames as F
    from metalhuffman_amd.codec import Huffman
    for h, w, seed in [(256, 256, 1), (64, 512, 2), (1024, 256, 3)]:
        ef = mh.encode_frame(F.uniform_random(h, w, seed))
        assert ef.canon.min() == ef.canon.max() == 8
        t1, t2 = Huffman.generateSplitLookupTables(ef.canon)
        o1, _ = oracle.split_tables(ef.canon)
        assert np.array_equal(t1, o1)
        pairs = t1.reshape(256, 2)
        assert np.array_equal(pairs[:, 0], np.arange(256)) and (pairs[:, 1] == 8).all()
