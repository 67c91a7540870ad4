"""GPU encoder (mh_encode_frame_device) vs the host codec, which is byte-identical to
the reference encoder (test_codec_parity.py, golden.json): canonical header, code
bytes (incl. the 4 zero pad bytes), block offsets and init bytes must match exactly,
and the GPU decoder must take the GPU-encoded frame back to the input."""
from __future__ import annotations

import numpy as np
import pytest

from helpers import fibonacci_deltas, image_from_block_deltas

pytestmark = pytest.mark.gpu


def _check(mh, device, img, flags=0, init_zero=False):
    import torch
    from metalhuffman_amd import decoder as D
    from metalhuffman_amd.encoder import encode_frame_device
    host = mh.encode_frame(img, flags=flags, init_zero_delta=init_zero)
    dev = encode_frame_device(torch.from_numpy(np.ascontiguousarray(img)).to(device), flags, init_zero)
    torch.cuda.synchronize(device)
    assert np.array_equal(dev.canon, host.canon)
    assert dev.codes.numel() == host.codes.size
    assert np.array_equal(dev.codes.cpu().numpy(), host.codes)
    assert np.array_equal(dev.block_offsets.cpu().numpy().view(np.uint32), host.block_offsets)
    if init_zero:
        assert np.array_equal(dev.block_init.cpu().numpy(), host.block_init)
    t1, t2 = mh.Huffman.generateSplitLookupTables(dev.canon)
    out = D.decode(dev.frames(), D.DeviceTables.upload(t1, t2, device))
    torch.cuda.synchronize(device)
    assert np.array_equal(out[0, :, : img.shape[1]].cpu().numpy(), img)


def test_encode_bigbridge(mh, device, bigbridge):
    _check(mh, device, bigbridge)


@pytest.mark.parametrize("hw", [(1, 1), (3, 5), (9, 17), (1001, 777), (8, 4096)])
def test_encode_odd_sizes(mh, device, bigbridge, hw):
    h, w = hw
    _check(mh, device, np.ascontiguousarray(np.tile(bigbridge, (1, 2))[:h, :w]))


def test_encode_random_and_variants(mh, device, bigbridge):
    from metalhuffman_amd import frames as F
    _check(mh, device, F.uniform_random(512, 512, 1234))
    _check(mh, device, np.ascontiguousarray(bigbridge[:768, :1024]), init_zero=True)
    d = fibonacci_deltas(15, 256 * 256, seed=4)
    _check(mh, device, image_from_block_deltas(d, 256, 256))                 # 14-bit codes
    _check(mh, device, fibonacci_deltas(17, 256 * 256, seed=3).reshape(256, 256), flags=1)


def test_encode_8192_tile(mh, device, bigbridge):
    from metalhuffman_amd import frames as F
    _check(mh, device, F.mirror_tile(bigbridge, 8192, 8192))


def test_encode_too_long_code_is_rejected(mh, device):
    import torch
    from metalhuffman_amd.encoder import encode_frame_device
    img = image_from_block_deltas(fibonacci_deltas(18, 256 * 256, seed=1), 256, 256)
    with pytest.raises(mh.MHError) as ei:
        encode_frame_device(torch.from_numpy(img).to(device))
    assert ei.value.status == -3
