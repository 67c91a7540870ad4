"""Batched GPU encoder (mh_encode_frames_device_async): n frames in
three launches, each frame with its own histogram, tree and codes, byte-identical
frame by frame to the host codec (itself byte-identical to the reference encoder,
Shared/HuffmanEncoder.cpp:310-381 / HuffmanUtil.cpp:1051-1131, golden.json), and
decodable as one batch when the frames share a table."""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

from helpers import fibonacci_deltas, golden, image_from_block_deltas

pytestmark = pytest.mark.gpu


def _check_batch(mh, device, imgs, flags=0, init_zero=False, expect_bad=()):
    import torch
    from metalhuffman_amd.encoder import BatchEncoder
    h, w = imgs[0].shape
    enc = BatchEncoder(w, h, len(imgs), device)
    grays = torch.from_numpy(np.ascontiguousarray(np.stack(imgs))).to(device)
    outs = []
    for _ in range(2):  # the workspace is reused: the second call must not see the first
        outs.append(enc.encode_async(grays, flags, init_zero))
    torch.cuda.synchronize(device)
    for a in outs:
        st = a.status.cpu().numpy()
        for f, img in enumerate(imgs):
            if f in expect_bad:
                assert st[f] == -3, (f, st[f])  # MH_ERR_CODE_TOO_LONG
                assert int(a.codes_len[f].item()) == 0
                continue
            assert st[f] == 0, (f, st[f])
            ref = mh.encode_frame(img, flags=flags, init_zero_delta=init_zero)
            r = a.frame(f)
            assert np.array_equal(r.canon, ref.canon), f
            assert r.codes.numel() == ref.codes.size, f
            assert np.array_equal(r.codes.cpu().numpy(), ref.codes), f
            assert np.array_equal(r.block_offsets.cpu().numpy().view(np.uint32), ref.block_offsets), f
            if init_zero:
                assert np.array_equal(r.block_init.cpu().numpy(), ref.block_init), f
        assert np.array_equal(a.frame_code_offsets.cpu().numpy(), np.arange(len(imgs) + 1) * a.slot)
    return outs[-1]


def test_batch_64_bigbridge_shuffles_decode_as_one_batch(mh, device, bigbridge):
    """The config-4 shard: 64 block-shuffled BigBridge frames encoded in one call,
    byte-identical to the host codec, then decoded in ONE launch with the shared table
    straight from the encoder's device slots (no host round trip)."""
    import torch
    from metalhuffman_amd import decoder as D
    from metalhuffman_amd import frames as F
    imgs = [F.block_shuffle(bigbridge, 300 + k) for k in range(64)]
    a = _check_batch(mh, device, imgs)
    canon = a.canon.cpu().numpy()
    assert all(np.array_equal(canon[0], c) for c in canon)  # block shuffles share the table
    t1, t2 = mh.Huffman.generateSplitLookupTables(canon[0])
    fr = a.frames()
    assert fr.code_bytes == int(a.codes_len.sum().item()) - 64 * mh.MH_CODES_PAD  # payload bytes
    out = D.decode(fr, D.DeviceTables.upload(t1, t2, device))
    torch.cuda.synchronize(device)
    assert torch.equal(out[..., :2048], torch.from_numpy(np.stack(imgs)).to(device))


def test_batch_pinned_to_reference_encoder_hashes(mh, device, bigbridge):
    """Frames pinned DIRECTLY to the reference encoder's output hashes (golden.json):
    BigBridge and its seed-7 block shuffle in one batch."""
    from metalhuffman_amd import frames as F
    g = golden()["workloads"]
    imgs = [bigbridge, F.block_shuffle(bigbridge, 7), bigbridge]
    a = _check_batch(mh, device, imgs)
    sha = lambda b: hashlib.sha256(np.ascontiguousarray(b).tobytes()).hexdigest()
    for f, wl in enumerate(["bigbridge", "bigbridge_shuffle_seed7", "bigbridge"]):
        rec = g[wl]
        r = a.frame(f)
        assert sha(r.canon) == rec["canon_sha256"]
        assert sha(r.codes.cpu().numpy()) == rec["huffbuff_sha256"]
        assert sha(r.block_offsets.cpu().numpy().view(np.uint32).astype("<u4")) == rec["offsets_sha256"]


def test_batch_mixed_histograms_and_rejected_frame(mh, device, bigbridge):
    """Frames with unrelated histograms in one batch (natural crop, uniform random,
    14-bit Fibonacci codes, a two-symbol frame) and one rejected frame (depth 17):
    every valid frame is exact, the rejected one reports MH_ERR_CODE_TOO_LONG and
    writes nothing, and no frame's tree leaks into another's."""
    from metalhuffman_amd import frames as F
    h, w = 256, 256
    imgs = [np.ascontiguousarray(bigbridge[:h, 500:500 + w]),
            F.uniform_random(w, h, 5),
            image_from_block_deltas(fibonacci_deltas(15, h * w, seed=4), w, h),
            image_from_block_deltas(fibonacci_deltas(19, h * w, seed=2), w, h),  # depth > 16
            np.where(np.arange(h * w).reshape(h, w) % 3 == 0, 7, 0).astype(np.uint8)]
    a = _check_batch(mh, device, imgs, expect_bad=(3,))
    # a batch holding a rejected frame is not handed to decode silently
    with pytest.raises(mh.MHError):
        a.frames()
    fr = a.frames(check=False)  # asynchronous: code_bytes is the slots' capacity
    assert fr.code_bytes == a.codes.numel() - len(imgs) * mh.MH_CODES_PAD


@pytest.mark.parametrize("hw", [(1, 1), (9, 17), (1001, 777), (8, 4096), (2056, 2048),
                                (64, 776), (72, 24), (80, 48), (136, 1032)])
def test_batch_odd_sizes_and_variants(mh, device, bigbridge, hw):
    """Partial edge blocks, one-block frames, tile counts that are not a multiple of
    the tile-offset chunk or of the packer's four waves per workgroup, frames larger than
    the single-frame fused path; every packer row loader: byte loads (W % 8 != 0), one
    8-byte load per block (W % 8 == 0 with an odd width in blocks: 776, 24, 1032), one
    16-byte load per block pair (an even width in blocks, narrower than a step: 48); the
    init-byte and no-delta formats."""
    from metalhuffman_amd import frames as F
    h, w = hw
    src = np.tile(bigbridge, (2, 2))
    imgs = [np.ascontiguousarray(F.block_shuffle(src, 11 + k)[:h, :w]) if h * w >= 64 else
            np.ascontiguousarray(src[k:k + h, :w]) for k in range(3)]
    _check_batch(mh, device, imgs)
    _check_batch(mh, device, imgs, init_zero=True)
    if h * w >= 4096:
        raw = [fibonacci_deltas(12, 64 * 64, seed=k).reshape(64, 64) for k in range(3)]
        _check_batch(mh, device, raw, flags=1)


def test_batch_unzeroed_workspace(mh, device, bigbridge):
    """Without MH_ENCODE_WORKSPACE_ZEROED the call zeroes the histograms itself: a
    workspace full of garbage still encodes exactly."""
    import ctypes

    import torch
    from metalhuffman_amd import _native as N
    from metalhuffman_amd import frames as F
    from metalhuffman_amd.encoder import BatchEncoder
    imgs = [np.ascontiguousarray(F.block_shuffle(bigbridge, 50 + k)[:512, :768]) for k in range(3)]
    enc = BatchEncoder(768, 512, 3, device)
    enc.workspace.fill_(0xA5)
    g = torch.from_numpy(np.stack(imgs)).to(device)
    n, nb = 3, enc.nb
    codes = torch.zeros(n * enc.slot + 16, dtype=torch.uint8, device=device)
    cb = (codes.data_ptr() + 15) // 16 * 16
    offs = torch.empty(n * nb, dtype=torch.int32, device=device)
    canon = torch.empty((n, 256), dtype=torch.uint8, device=device)
    lens = torch.empty(n, dtype=torch.int64, device=device)
    st = torch.empty(n, dtype=torch.int32, device=device)
    base = enc.workspace.data_ptr()
    al = (base + 255) // 256 * 256
    N.check(N.lib().mh_encode_frames_device_async(
        g.data_ptr(), 768 * 512, n, 768, 512, 0, canon.data_ptr(), cb, enc.slot, lens.data_ptr(), None,
        offs.data_ptr(), None, st.data_ptr(), al, enc.workspace.numel() - (al - base),
        ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)), "batch")
    torch.cuda.synchronize(device)
    host = codes.cpu().numpy()[cb - codes.data_ptr():]
    for f, img in enumerate(imgs):
        ref = mh.encode_frame(img)
        assert int(st[f].item()) == 0
        assert int(lens[f].item()) == ref.codes.size
        assert np.array_equal(canon[f].cpu().numpy(), ref.canon)
        assert np.array_equal(host[f * enc.slot: f * enc.slot + ref.codes.size], ref.codes)
        assert np.array_equal(offs[f * nb:(f + 1) * nb].cpu().numpy().view(np.uint32), ref.block_offsets)


def test_batch_argument_checks(mh, device):
    """Misaligned slots, zero frames and bad flags are refused before any launch."""
    import torch
    from metalhuffman_amd import _native as N
    L = N.lib()
    ws = torch.zeros(int(L.mh_encode_frames_workspace_bytes(64, 64, 2)) + 256, dtype=torch.uint8, device=device)
    al = (ws.data_ptr() + 255) // 256 * 256
    buf = torch.zeros(1 << 16, dtype=torch.uint8, device=device)
    p = (buf.data_ptr() + 255) // 256 * 256
    args = lambda n, stride, flags, codes: (p, 64 * 64, n, 64, 64, flags, p, codes, stride, None, None, p, None, None,
                                            al, ws.numel() - 256, None)
    assert L.mh_encode_frames_device_async(*args(0, 1024, 0, p)) == -1  # MH_ERR_INVALID_ARG
    assert L.mh_encode_frames_device_async(*args(2, 1000, 0, p)) == -6  # MH_ERR_ALIGN
    assert L.mh_encode_frames_device_async(*args(2, 1024, 0, p + 4)) == -6
    assert L.mh_encode_frames_device_async(*args(2, 1024, 0x40, p)) == -1
