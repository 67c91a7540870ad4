"""Time-boxed randomized GPU parity sweep (MH_STRESS_SECONDS, default 15 s).

Each case is generated from its index alone (seeded), so a failure names a case that
replays exactly. Every case: the product's host codec encodes a generated frame
(byte-identical to the reference encoder, test_codec_parity.py); the GPU decodes it
through the C-ABI and must return the input. Every 8th case (up to 1 Mpixel) is also
compared with the oracle's shader-semantics decode, every 4th case's GPU encoder
output (header, code bytes, block offsets, init bytes) with the host codec's, and
every batch of frames sharing a table is also GPU-encoded in one batched call
(mh_encode_frames_device_async) and compared frame by frame.

Frame kinds: natural-like (geometric steps), Gaussian noise, uniform bytes, sparse
alphabets (2-6 symbols), a constant frame (one-symbol alphabet), Fibonacci histograms
(13-16-bit codes), BigBridge crops with shuffled blocks, ramps. Formats: deltas, no
deltas, per-block init byte. Paths: single-frame launch with the prepared table (the
small kernel), with the in-kernel table (the batch kernel), batches of 2-6 frames
sharing one table, the lane-pair variant, any-order launches.
"""
from __future__ import annotations

import os
import time

import numpy as np
import pytest

from helpers import fibonacci_deltas, image_from_block_deltas

pytestmark = pytest.mark.gpu

KINDS = ("geometric", "normal", "uniform", "sparse", "constant", "fibonacci", "bigbridge", "ramp")
MODES = ("prepared", "in_kernel", "batch", "lane_pairs", "any_order")


def _frame(case: int, bigbridge: np.ndarray):
    r = np.random.default_rng(1_000_003 * case + 17)
    kind = KINDS[case % len(KINDS)]
    big = r.random() < 0.08
    h = int(r.integers(1, 4097 if big else 1201))
    w = int(r.integers(1, 4097 if big else 1201))
    if kind == "geometric":
        img = np.minimum(r.geometric(r.uniform(0.05, 0.7), size=(h, w)) - 1, 255).astype(np.uint8)
        img = np.cumsum(img, axis=int(r.integers(0, 2)), dtype=np.uint8)
    elif kind == "normal":
        img = (np.round(r.normal(int(r.integers(0, 256)), r.uniform(0.5, 40), size=(h, w))) % 256).astype(np.uint8)
    elif kind == "uniform":
        img = r.integers(0, 256, size=(h, w), dtype=np.uint8)
    elif kind == "sparse":
        alpha = r.choice(256, size=int(r.integers(2, 7)), replace=False).astype(np.uint8)
        img = alpha[r.integers(0, alpha.size, size=(h, w))]
    elif kind == "constant":
        img = np.full((h, w), int(r.integers(0, 256)), np.uint8)
    elif kind == "fibonacci":
        h, w = max(8, h // 8 * 8), max(8, w // 8 * 8)
        n_sym = int(r.integers(12, 18))  # deepest code n_sym - 1 bits: 11..16
        img = image_from_block_deltas(fibonacci_deltas(n_sym, h * w, seed=case), w, h)
    elif kind == "bigbridge":
        h, w = min(h, bigbridge.shape[0]), min(w, bigbridge.shape[1])
        y = int(r.integers(0, bigbridge.shape[0] - h + 1))
        x = int(r.integers(0, bigbridge.shape[1] - w + 1))
        img = np.ascontiguousarray(bigbridge[y:y + h, x:x + w])
        if h % 8 == 0 and w % 8 == 0 and r.random() < 0.5:
            from metalhuffman_amd import frames as F
            img = F.block_shuffle(img, case)
    else:  # ramp
        yy, xx = np.mgrid[0:h, 0:w]
        img = ((yy * int(r.integers(0, 5)) + xx * int(r.integers(0, 5))) % 256).astype(np.uint8)
    fmt = int(r.integers(0, 3))
    mode = MODES[int(r.integers(0, len(MODES)))]
    return kind, np.ascontiguousarray(img), fmt, mode


def test_randomized_parity_sweep(mh, oracle, device, bigbridge):
    import torch
    from metalhuffman_amd import _native as N
    from metalhuffman_amd import decoder as D
    from metalhuffman_amd import frames as F
    from metalhuffman_amd.encoder import BatchEncoder, encode_frame_device

    budget = float(os.environ.get("MH_STRESS_SECONDS", "15"))
    first = int(os.environ.get("MH_STRESS_FIRST_CASE", "0"))
    t_end = time.perf_counter() + budget
    stats = {"cases": 0, "rejected": 0, "oracle": 0, "encoder": 0, "batch_encoder": 0, "pixels": 0}
    per_mode = dict.fromkeys(MODES, 0)
    case = first
    last_report = time.perf_counter()
    while time.perf_counter() < t_end or stats["cases"] < 8:
        kind, img, fmt, mode = _frame(case, bigbridge)
        h, w = img.shape
        kw = {"flags": mh.MH_FLAG_NO_DELTA} if fmt == 1 else ({"init_zero_delta": True} if fmt == 2 else {})
        try:
            ef = mh.encode_frame(img, **kw)
        except mh.MHError:
            stats["rejected"] += 1  # a code deeper than 16 bits: invalid for the reference too
            case += 1
            continue
        tag = (case, kind, h, w, fmt, mode)
        t1, t2 = ef.tables()
        tabs = D.DeviceTables.upload(t1, t2, device, prepare_lut=(mode != "in_kernel"))
        ref = torch.from_numpy(img).to(device)
        if mode == "batch" and h % 8 == 0 and w % 8 == 0:
            # frames sharing one table: block shuffles keep the histogram
            n = int(np.random.default_rng(case).integers(2, 7))
            imgs = [img] + [F.block_shuffle(img, 10_000 + case * 8 + k) for k in range(n - 1)]
            efs = [ef] + [mh.encode_frame(im, **kw) for im in imgs[1:]]
            assert all(np.array_equal(e.canon, ef.canon) for e in efs), tag
            out = D.decode(D.DeviceFrames.pack(efs, device), tabs)
            refs = torch.from_numpy(np.stack(imgs)).to(device)
            torch.cuda.synchronize(device)
            bad = [i for i in range(n) if not torch.equal(out[i, :, :w], refs[i])]
            assert not bad, (tag, bad)
            # the batched GPU encoder on the same frames: byte-identical frame by frame
            benc = BatchEncoder(w, h, n, device)
            a = benc.encode_async(refs, ef.flags & 1, fmt == 2)
            torch.cuda.synchronize(device)
            for i, e in enumerate(efs):
                r = a.frame(i)
                assert int(a.status[i].item()) == 0, (tag, i)
                assert np.array_equal(r.canon, e.canon), (tag, i)
                assert np.array_equal(r.codes.cpu().numpy(), e.codes), (tag, i)
                assert np.array_equal(r.block_offsets.cpu().numpy().view(np.uint32), e.block_offsets), (tag, i)
                if fmt == 2:
                    assert np.array_equal(r.block_init.cpu().numpy(), e.block_init), (tag, i)
            stats["batch_encoder"] += n
        elif mode == "any_order":
            frs = D.DeviceFrames.pack([ef], device)
            outs = [D.decode(frs, tabs, extra_flags=N.MH_FLAG_ANY_ORDER if k else 0) for k in range(3)]
            torch.cuda.synchronize(device)
            assert all(torch.equal(o[0, :, :w], ref) for o in outs), tag
        else:
            extra = N.MH_FLAG_LANE_PAIRS if mode == "lane_pairs" else 0
            out = D.decode(D.DeviceFrames.pack([ef], device), tabs, extra_flags=extra)
            torch.cuda.synchronize(device)
            assert torch.equal(out[0, :, :w], ref), tag
            if case % 8 == 0 and h * w <= (1 << 20):
                o = oracle.decode_frame_shader(ef.block_offsets, ef.codes, t1, t2, w, h,
                                               block_init=ef.block_init, delta=not (ef.flags & 1))
                assert np.array_equal(out[0, :, :w].cpu().numpy(), o), tag
                stats["oracle"] += 1
        if case % 4 == 0:
            dev = encode_frame_device(ref, ef.flags & 1, fmt == 2)
            torch.cuda.synchronize(device)
            assert np.array_equal(dev.canon, ef.canon), tag
            assert np.array_equal(dev.codes.cpu().numpy(), ef.codes), tag
            assert np.array_equal(dev.block_offsets.cpu().numpy().view(np.uint32), ef.block_offsets), tag
            if fmt == 2:
                assert np.array_equal(dev.block_init.cpu().numpy(), ef.block_init), tag
            stats["encoder"] += 1
        stats["cases"] += 1
        stats["pixels"] += h * w
        per_mode[mode] += 1
        case += 1
        if time.perf_counter() - last_report > 10:
            last_report = time.perf_counter()
            print(f"[stress] {stats} modes {per_mode}", flush=True)
    print(f"[stress] done: cases {first}..{case - 1} {stats} modes {per_mode}", flush=True)
    assert stats["cases"] >= 8
