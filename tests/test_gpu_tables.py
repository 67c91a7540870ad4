"""GPU-side table build from the 256-byte canonical header (mh_build_tables_device)
against the host builder (itself byte-identical to the reference's split tables,
test_codec_parity.py): T1, T2, the used entry count and the prepared decode table
must match byte for byte, and decoding through device-built tables is exact."""
from __future__ import annotations

import os

import numpy as np
import pytest

from helpers import GOLDEN, fibonacci_deltas, golden, image_from_block_deltas

pytestmark = pytest.mark.gpu


def _headers(mh, bigbridge):
    from metalhuffman_amd import frames as F
    out = {"bigbridge": mh.encode_frame(bigbridge).canon,
           "random1024": mh.encode_frame(F.uniform_random(1024, 1024, 1234)).canon,
           "single": mh.encode_frame(np.zeros((16, 16), np.uint8)).canon,
           "empty": np.zeros(256, np.uint8)}
    for n in (14, 15, 17):
        d = fibonacci_deltas(n, 256 * 256, seed=n)
        out[f"fib{n}"] = mh.encode_frame(image_from_block_deltas(d, 256, 256)).canon
    for name, fx in golden()["small_frames"].items():
        c = np.zeros(256, np.uint8)
        for k, v in fx["canon"].items():
            c[int(k)] = v
        out[name] = c
    from PIL import Image
    gray = np.array(Image.open(os.path.join(GOLDEN, "Image.png")).convert("L"), np.uint8)
    out["image512"] = mh.encode_frame(gray).canon
    return out


def test_device_tables_match_host_builder(mh, device, bigbridge):
    import torch
    from metalhuffman_amd import decoder as D
    for name, canon in _headers(mh, bigbridge).items():
        t1, t2 = mh.Huffman.generateSplitLookupTables(canon)
        dev = D.DeviceTables.from_canonical_header(canon, device)
        entries = dev.check_status()
        assert entries * 2 == t2.size, name
        assert np.array_equal(dev.table1.cpu().numpy(), t1), name
        d2 = dev.table2.cpu().numpy()
        assert np.array_equal(d2[: t2.size], t2), name
        assert not d2[t2.size:].any(), name                      # zero past the used subtables
        host = D.DeviceTables.upload(t1, t2, device)            # mh_prepare_lut on uploaded tables
        torch.cuda.synchronize(device)
        assert np.array_equal(dev.lut.cpu().numpy(), host.lut.cpu().numpy()), name


def test_decode_through_device_built_tables(mh, device, bigbridge):
    import torch
    from metalhuffman_amd import decoder as D
    from metalhuffman_amd import frames as F
    imgs = [bigbridge] + [F.block_shuffle(bigbridge, s) for s in (3, 4)]
    efs = [mh.encode_frame(im) for im in imgs]
    tabs = D.DeviceTables.from_canonical_header(torch.from_numpy(efs[0].canon).to(device), device)
    for batch in ([efs[0]], efs):                                # small-launch and batch kernels
        out = D.decode(D.DeviceFrames.pack(batch, device), tabs)
        torch.cuda.synchronize(device)
        for i, ef in enumerate(batch):
            assert np.array_equal(out[i, :, : ef.width].cpu().numpy(), imgs[i]), i


@pytest.mark.parametrize("bad,status", [({7: 17}, -3), ({1: 1, 2: 1, 3: 1}, -5)])
def test_device_tables_reject_bad_headers(mh, device, bad, status):
    from metalhuffman_amd import decoder as D
    canon = np.zeros(256, np.uint8)
    for s, ln in bad.items():
        canon[s] = ln
    dev = D.DeviceTables.from_canonical_header(canon, device)
    with pytest.raises(mh.MHError) as ei:
        dev.check_status()
    assert ei.value.status == status
    assert not dev.table1.cpu().numpy().any()


def test_device_tables_random_headers(mh, device):
    """40 canonical headers from random histograms (short and long codes, a few
    symbols to all 256, lengths up to 16): T1, T2 and the prepared table built on the
    device equal the host builder + mh_prepare_lut byte for byte (the device derives
    P0 and the longest/shortest-code words from the canonical codes)."""
    import ctypes
    import torch
    from metalhuffman_amd import _native as N
    from metalhuffman_amd import decoder as D
    rng = np.random.default_rng(77)
    done = 0
    while done < 40:
        k = int(rng.integers(2, 257))
        f = np.zeros(256, np.uint64)
        syms = rng.choice(256, k, replace=False)
        f[syms] = np.round(2.0 ** rng.uniform(0, rng.uniform(2, 17), k)).astype(np.uint64)
        canon = np.zeros(256, np.uint8)
        if N.lib().mh_code_lengths(f.ctypes.data_as(N._u64p), canon.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))):
            continue  # depth > 16: not a valid header
        t1, t2 = mh.Huffman.generateSplitLookupTables(canon)
        dev = D.DeviceTables.from_canonical_header(canon, device)
        assert dev.check_status() * 2 == t2.size
        assert np.array_equal(dev.table1.cpu().numpy(), t1)
        d2 = dev.table2.cpu().numpy()
        assert np.array_equal(d2[: t2.size], t2) and not d2[t2.size:].any()
        host = D.DeviceTables.upload(t1, t2, device)
        torch.cuda.synchronize(device)
        assert np.array_equal(dev.lut.cpu().numpy(), host.lut.cpu().numpy()), (k, int(canon.max()))
        done += 1


def test_device_tables_bigbridge_golden_hashes(mh, device, bigbridge):
    """Device-built T1/T2 for BigBridge pinned to the recorded SHA-256 (SURVEY.md 8(c),
    golden.json), not only to the host builder."""
    import hashlib
    from metalhuffman_amd import decoder as D
    rec = golden()["workloads"]["bigbridge"]
    dev = D.DeviceTables.from_canonical_header(mh.encode_frame(bigbridge).canon, device)
    entries = dev.check_status()
    assert entries * 2 == rec["t2_bytes"]
    sha = lambda b: hashlib.sha256(np.ascontiguousarray(b).tobytes()).hexdigest()
    assert sha(dev.table1.cpu().numpy()) == rec["t1_sha256"]
    assert sha(dev.table2.cpu().numpy()[: rec["t2_bytes"]]) == rec["t2_sha256"]
