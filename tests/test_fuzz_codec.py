"""Property-based parity of the product's host side (csrc/mh_host.cpp, csrc/mh_cpu.cpp)
against the oracle, over generated frames: random W x H (ragged edge blocks), alphabet
sizes 1..256, skewed / smooth / uniform / constant value distributions and the
reference's format options (deltas off, AAPLShaderTypes.h:109; init-zero delta, :110).

Properties (CPU only, deterministic: hypothesis derandomised):
  * encode_frame is byte-identical to the oracle's restatement of HuffmanEncoder::encode
    + Util.m's split (canon, codes, block offsets), or both reject the frame
    (a code longer than 16 bits: MH_ERR_CODE_TOO_LONG, the reference's 16-bit limit);
  * the serial T1/T2 decoder (HuffmanUtil.cpp:830-1046) returns the oracle's symbols and
    bit offsets, and every 64th offset is the encoder's block offset;
  * the threaded frame decoder reproduces the input picture and the oracle's shader
    restatement (AAPLShaders.metal:241-268) for any thread count;
  * with oracle/_ref built (container only), the real reference encoder emits the same
    bytes for the split+delta symbol stream.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

hyp = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import event  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

from helpers import fibonacci_deltas, image_from_block_deltas  # noqa: E402

SETTINGS = dict(max_examples=300, deadline=None, derandomize=True,
                suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])


def _image(kind: str, seed: int) -> np.ndarray:
    """A generated frame. Size and alphabet come from the seed (uniform over 1..160 x
    1..120 and 1..256): hypothesis's own integers favour tiny values."""
    r = np.random.default_rng(seed)
    w, h, k = int(r.integers(1, 161)), int(r.integers(1, 121)), int(r.integers(1, 257))
    if kind == "const":
        return np.full((h, w), seed & 0xFF, np.uint8)
    if kind == "uniform":
        return r.integers(0, k, size=(h, w)).astype(np.uint8)
    if kind == "sparse":  # few distinct values spread over the byte range
        vals = r.choice(256, size=k, replace=False).astype(np.uint8)
        return vals[r.integers(0, k, size=(h, w))]
    if kind == "geometric":  # heavily skewed alphabet (long codes)
        return np.minimum(r.geometric(0.45, size=(h, w)) - 1, 255).astype(np.uint8)
    if kind == "fibonacci":  # deepest code 11..18 bits: past 16 both sides must reject
        # at least 128 x 96 pixels so that all 19 symbols of the deepest shape occur
        w8, h8 = max(-(-w // 8) * 8, 128), max(-(-h // 8) * 8, 96)
        d = fibonacci_deltas(12 + seed % 8, w8 * h8, seed=seed)
        return image_from_block_deltas(d, w8, h8)
    # smooth: a gradient plus small noise, like a photograph's deltas
    y, x = np.mgrid[0:h, 0:w]
    base = (x * (seed % 7 + 1) + y * (seed % 5)) // 3
    return ((base + r.integers(-k // 16 - 1, k // 16 + 2, size=(h, w))) & 0xFF).astype(np.uint8)


frames = st.tuples(
    st.sampled_from(["const", "uniform", "sparse", "geometric", "fibonacci", "smooth"]),
    st.integers(0, 2**31 - 1),  # seed: size, alphabet and values
)


@settings(**SETTINGS)
@given(frames, st.integers(1, 5))
def test_encode_decode_parity(mh, oracle, spec, threads):
    img = _image(*spec)
    h, w = img.shape
    try:
        want = oracle.encode_frame(img)
    except oracle.OracleError:
        event("both reject (code > 16 bits)")
        with pytest.raises(mh.MHError) as e:
            mh.encode_frame(img)
        assert e.value.status == -3  # MH_ERR_CODE_TOO_LONG
        return
    event(f"longest code {int(want[0].max())} bits")
    ef = mh.encode_frame(img)
    canon, huff, offs = want
    assert np.array_equal(ef.canon, canon)
    assert np.array_equal(ef.codes, huff)
    assert np.array_equal(ef.block_offsets, offs)

    t1, t2 = ef.tables()
    nsym = ef.n_blocks * 64
    sym, bits = oracle.decode_from_tables(t1, t2, nsym, ef.codes, want_offsets=True)
    got, gbits = mh.Huffman.decodeHuffmanBitsFromTables(t1, t2, 8, 8, nsym, ef.codes, bitOffsets=True)
    assert np.array_equal(got, sym) and np.array_equal(gbits, bits)
    assert np.array_equal(gbits[::64], ef.block_offsets)

    out = mh.decode_frame_cpu(ef, threads)
    assert np.array_equal(out, img)
    assert np.array_equal(out, oracle.decode_frame_shader(ef.block_offsets, ef.codes, t1, t2, w, h))


@settings(**SETTINGS)
@given(frames, st.sampled_from(["no_delta", "init_zero"]), st.integers(1, 4))
def test_format_options(mh, oracle, spec, option, threads):
    img = _image(*spec)
    h, w = img.shape
    try:
        if option == "no_delta":
            ef = mh.encode_frame(img, flags=mh.MH_FLAG_NO_DELTA)
        else:
            ef = mh.encode_frame(img, init_zero_delta=True)
    except mh.MHError as e:
        assert e.status == -3
        event("rejected (code > 16 bits)")
        return
    t1, t2 = ef.tables()
    ref = oracle.decode_frame_shader(ef.block_offsets, ef.codes, t1, t2, w, h,
                                     block_init=ef.block_init, delta=option != "no_delta")
    out = mh.decode_frame_cpu(ef, threads)
    assert np.array_equal(out, ref)
    assert np.array_equal(out, img)


@pytest.mark.ref
@pytest.mark.skipif(not os.path.isdir("/root/reference/Shared"), reason="needs /root/reference")
@settings(**{**SETTINGS, "max_examples": 100})
@given(frames)
def test_reference_encoder_agrees(mh, oracle, spec):
    """The real reference encoder (compiled from /root/reference into oracle/_ref) on
    the split + delta symbols of the generated frame."""
    if not os.path.exists(oracle.REF_ENCODE) and not oracle.build_ref():
        pytest.skip("reference encoder not buildable")
    img = _image(*spec)
    sym = oracle.delta_encode(oracle.split_blocks(img))
    try:
        canon, codes, offs = oracle.huffman_encode(sym, 64)
    except oracle.OracleError:
        event("code > 16 bits (the reference asserts)")
        return  # code too long: the reference asserts (aborts) here
    event("reference encoder ran")
    c2, k2, o2 = oracle.ref_encode(sym, 64)
    assert np.array_equal(canon, c2) and np.array_equal(codes, k2) and np.array_equal(offs, o2)
