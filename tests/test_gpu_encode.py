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


@pytest.mark.parametrize("hw", [(2048, 2048), (2056, 2048), (8, 65528), (2048, 1536)])
def test_async_encode_fused_path_boundary(mh, device, bigbridge, hw):
    """Frames of up to 512 tiles of 128 blocks take the two-launch path (tiled split +
    code kernel), larger ones the four-kernel path. (h, w) = (2048, 2048) is exactly
    512 tiles, (2056, 2048) 514, (8, 65528) one block row of 8191 blocks (64 tiles,
    the last partial), (2048, 1536) BigBridge's shape transposed. Both sides
    byte-identical to the host codec."""
    from metalhuffman_amd import frames as F
    h, w = hw
    img = np.ascontiguousarray(F.mirror_tile(bigbridge, h, w)) if h > 8 else \
        np.ascontiguousarray(np.tile(bigbridge[:8], (1, w // bigbridge.shape[1] + 1))[:, :w])
    _check_async(mh, device, img)


def test_encode_too_long_code_is_rejected(mh, device):
    import torch
    from metalhuffman_amd.encoder import encode_frame_device
    img = image_from_block_deltas(fibonacci_deltas(18, 256 * 256, seed=1), 256, 256)
    with pytest.raises(mh.MHError) as ei:
        encode_frame_device(torch.from_numpy(img).to(device))
    assert ei.value.status == -3


# ---- mh_encode_frame_device_async: the tree on the device, no host sync ----

def _check_async(mh, device, img, flags=0, init_zero=False):
    import torch
    from metalhuffman_amd import decoder as D
    from metalhuffman_amd.encoder import Encoder
    host = mh.encode_frame(img, flags=flags, init_zero_delta=init_zero)
    h, w = img.shape
    enc = Encoder(w, h, device)
    a = enc.encode_async(torch.from_numpy(np.ascontiguousarray(img)).to(device), flags, init_zero)
    # decode straight from the device header and the whole code buffer, then look
    out = D.decode(a.frames(), a.tables())
    torch.cuda.synchronize(device)
    assert int(a.status.item()) == 0
    assert int(a.codes_len.item()) == host.codes.size
    assert np.array_equal(a.canon.cpu().numpy(), host.canon)
    assert np.array_equal(a.codes[: host.codes.size].cpu().numpy(), host.codes)
    assert np.array_equal(a.block_offsets.cpu().numpy().view(np.uint32), host.block_offsets)
    if init_zero:
        assert np.array_equal(a.block_init.cpu().numpy(), host.block_init)
    assert np.array_equal(out[0, :, :w].cpu().numpy(), img)
    r = a.result()
    assert r.codes.numel() == host.codes.size and np.array_equal(r.canon, host.canon)


def test_async_encode_bigbridge_and_variants(mh, device, bigbridge):
    from metalhuffman_amd import frames as F
    _check_async(mh, device, bigbridge)
    _check_async(mh, device, np.ascontiguousarray(bigbridge[:777, :1001]), init_zero=True)
    _check_async(mh, device, F.uniform_random(256, 320, 77))
    _check_async(mh, device, fibonacci_deltas(17, 128 * 128, seed=8).reshape(128, 128), flags=1)
    _check_async(mh, device, np.full((9, 17), 200, np.uint8))          # one delta symbol (0)
    _check_async(mh, device, np.full((16, 16), 7, np.uint8), flags=1)   # one raw symbol


def _deltas_with_histogram(counts: np.ndarray, seed: int) -> np.ndarray:
    d = np.repeat(np.arange(256, dtype=np.uint8), counts.astype(np.int64))
    np.random.default_rng(seed).shuffle(d)
    return d


@pytest.mark.parametrize("seed", range(6))
def test_async_tree_matches_reference_tie_breaking(mh, device, seed):
    """Histograms full of equal weights (where the reference's upper_bound insertion
    decides the tree), random small counts and a Fibonacci-like ladder up to depth
    16: the device tree must give the host codec's header (mh_code_lengths, pinned
    to the reference encoder) byte for byte."""
    rng = np.random.default_rng(100 + seed)
    k = int(rng.integers(2, 257))
    syms = rng.choice(256, k, replace=False)
    counts = np.zeros(256, np.int64)
    kind = seed % 3
    if kind == 0:
        counts[syms] = 64                               # all equal
    elif kind == 1:
        counts[syms] = rng.integers(1, 6, k) * 8        # many ties
    else:
        fib = [1, 1]
        while len(fib) < min(k, 16):
            fib.append(fib[-1] + fib[-2])
        counts[syms[: len(fib)]] = np.array(fib) * 8
        counts[syms[len(fib):]] = 8
    total = int(counts.sum())
    side = 8 * int(np.ceil(np.sqrt(total / 64.0)))
    counts[syms[0]] += side * side - total             # pad to a whole square of blocks
    d = _deltas_with_histogram(counts, seed)
    img = image_from_block_deltas(d, side, side)
    _check_async(mh, device, img)


def test_async_encode_errors_write_nothing(mh, device):
    import torch
    from metalhuffman_amd.encoder import Encoder
    img = image_from_block_deltas(fibonacci_deltas(18, 256 * 256, seed=1), 256, 256)
    enc = Encoder(256, 256, device)
    codes = torch.full((enc.cap,), 0xAB, dtype=torch.uint8, device=device)
    a = enc.encode_async(torch.from_numpy(img).to(device), codes=codes)
    torch.cuda.synchronize(device)
    assert int(a.status.item()) == -3 and int(a.codes_len.item()) == 0
    assert bool((codes == 0xAB).all())
    with pytest.raises(mh.MHError):
        a.result()
    # a code buffer too small for the frame: MH_ERR_CAPACITY on the device
    from metalhuffman_amd import frames as F
    small = torch.full((1024,), 0xCD, dtype=torch.uint8, device=device)
    b = enc.encode_async(torch.from_numpy(F.uniform_random(256, 256, 5)).to(device), codes=small)
    torch.cuda.synchronize(device)
    assert int(b.status.item()) == -4 and int(b.codes_len.item()) == 0
    assert bool((small == 0xCD).all())


def test_async_encode_many_frames_back_to_back(mh, device, bigbridge):
    """Frames enqueued back to back on one workspace (the scan's completion ticket and
    the histograms are reused every call), then on two streams with one encoder each:
    every frame byte-identical to the host codec."""
    import torch
    from metalhuffman_amd import frames as F
    from metalhuffman_amd.encoder import Encoder
    h, w = 512, 768
    imgs = [np.ascontiguousarray(F.block_shuffle(bigbridge, 40 + k)[:h, :w]) for k in range(24)]
    hosts = [mh.encode_frame(im) for im in imgs]
    dimgs = [torch.from_numpy(im).to(device) for im in imgs]
    enc = Encoder(w, h, device)
    outs = [enc.encode_async(d) for d in dimgs]
    encs = [Encoder(w, h, device) for _ in range(2)]
    streams = [torch.cuda.Stream(device) for _ in range(2)]
    for st in streams:  # the frames were uploaded on the current stream
        st.wait_stream(torch.cuda.current_stream(device))
    outs2 = [encs[k % 2].encode_async(d, stream=streams[k % 2]) for k, d in enumerate(dimgs)]
    torch.cuda.synchronize(device)
    for o, o2, ref in zip(outs, outs2, hosts):
        for a in (o, o2):
            r = a.result()
            assert np.array_equal(r.canon, ref.canon)
            assert np.array_equal(r.codes.cpu().numpy(), ref.codes)
            assert np.array_equal(r.block_offsets.cpu().numpy().view(np.uint32), ref.block_offsets)


def test_async_encode_fuzz_shapes_and_histograms(mh, device):
    """Random sizes (partial blocks included) and random delta histograms, from a
    few symbols to all 256 and codes up to 16 bits: the device tree, codes and
    offsets equal the host codec's, and the device-only decode returns the frame."""
    rng = np.random.default_rng(2024)
    done = 0
    while done < 16:
        h, w = int(rng.integers(1, 300)), int(rng.integers(1, 300))
        k = int(rng.integers(1, 257))
        syms = rng.choice(256, k, replace=False)
        p = 2.0 ** rng.uniform(0, rng.uniform(1, 14), k)
        nb = ((w + 7) // 8) * ((h + 7) // 8)
        d = rng.choice(syms, size=nb * 64, p=p / p.sum()).astype(np.uint8)
        bw = (w + 7) // 8
        img = image_from_block_deltas(d, bw * 8, nb // bw * 8)[:h, :w]
        try:
            mh.encode_frame(img)
        except mh.MHError:
            continue  # depth > 16 after the crop's zero padding: not a valid frame
        _check_async(mh, device, np.ascontiguousarray(img))
        done += 1


@pytest.mark.parametrize("wl", ["bigbridge", "bigbridge_crop_777x1001", "random_1024_seed1234",
                                "bigbridge_shuffle_seed7", "tile_8192"])
def test_device_encoder_matches_reference_encoder_hashes(mh, device, bigbridge, wl):
    """The device encoder pinned DIRECTLY to the reference encoder: SHA-256 of its
    canonical header, huffBuff (codes + zero pad) and block offsets equal those of
    Shared/HuffmanEncoder.cpp:310-381 compiled here (tests/golden/golden.json), not
    only the host codec's bytes."""
    import hashlib
    import torch
    from helpers import golden
    from metalhuffman_amd import frames as F
    from metalhuffman_amd.encoder import encode_frame_device
    rec = golden()["workloads"][wl]
    img = {"bigbridge": lambda: bigbridge,
           "bigbridge_crop_777x1001": lambda: F.crop(bigbridge, 1001, 777),
           "random_1024_seed1234": lambda: F.uniform_random(1024, 1024, 1234),
           "bigbridge_shuffle_seed7": lambda: F.block_shuffle(bigbridge, 7),
           "tile_8192": lambda: F.mirror_tile(bigbridge, 8192, 8192)}[wl]()
    sha = lambda b: hashlib.sha256(np.ascontiguousarray(b).tobytes()).hexdigest()
    assert sha(img) == rec["input_sha256"]
    dev = encode_frame_device(torch.from_numpy(np.ascontiguousarray(img)).to(device))
    torch.cuda.synchronize(device)
    assert sha(dev.canon) == rec["canon_sha256"]
    codes = dev.codes.cpu().numpy()
    assert codes.size == rec["huffbuff_bytes"]
    assert sha(codes) == rec["huffbuff_sha256"]
    assert sha(dev.block_offsets.cpu().numpy().view(np.uint32).astype("<u4")) == rec["offsets_sha256"]


def test_async_encode_workspace_flag(mh, device, bigbridge):
    """Without MH_ENCODE_WORKSPACE_ZEROED the call clears the histogram itself (a
    workspace full of garbage still encodes exactly); with it, a workspace that was
    zero-filled once stays valid call after call (each tree kernel re-zeroes the
    histogram it consumed), including after a rejected frame."""
    import ctypes
    import torch
    from metalhuffman_amd import _native as N
    from metalhuffman_amd.encoder import Encoder
    from metalhuffman_amd import frames as F
    h, w = 512, 768
    img = np.ascontiguousarray(F.block_shuffle(bigbridge, 40)[:h, :w])
    ref = mh.encode_frame(img)
    enc = Encoder(w, h, device)
    d = torch.from_numpy(img).to(device)
    enc.workspace.fill_(0xFF)
    codes = torch.empty(enc.cap, dtype=torch.uint8, device=device)
    offs = torch.empty(enc.nb, dtype=torch.int32, device=device)
    canon = torch.empty(256, dtype=torch.uint8, device=device)
    meta = torch.zeros(2, dtype=torch.int64, device=device)
    base = enc.workspace.data_ptr()
    aligned = (base + 255) // 256 * 256
    N.check(N.lib().mh_encode_frame_device_async(
        d.data_ptr(), w, h, 0, canon.data_ptr(), codes.data_ptr(), codes.numel(), meta.data_ptr(),
        offs.data_ptr(), None, meta.data_ptr() + 8, aligned, enc.workspace.numel() - (aligned - base),
        ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)), "mh_encode_frame_device_async")
    torch.cuda.synchronize(device)
    n = int(meta[0].item())
    assert np.array_equal(canon.cpu().numpy(), ref.canon)
    assert np.array_equal(codes[:n].cpu().numpy(), ref.codes)
    # the flag path (Encoder): zero-filled once, then frames, a rejected one, frames
    enc2 = Encoder(w, h, device)
    bad = torch.from_numpy(image_from_block_deltas(fibonacci_deltas(18, h * w, seed=2), w, h)).to(device)
    for k, g in enumerate([d, bad, d, d]):
        a = enc2.encode_async(g)
        torch.cuda.synchronize(device)
        if k == 1:
            assert int(a.status.item()) == -3
            continue
        r = a.result()
        assert np.array_equal(r.canon, ref.canon) and np.array_equal(r.codes.cpu().numpy(), ref.codes), k


@pytest.mark.parametrize("path", ["2"])
def test_fused_encoder_timeout_is_sticky(mh, path):
    """A packing workgroup that gives up waiting for the code table (diagnostic build
    with a zero spin budget, MH_DIAG_SPIN_TICKS=0) must leave MH_ERR_HIP in the status,
    whenever workgroup 0's own status store lands (mh_encode.hip: meta[kAbort], all
    four accesses sequentially consistent). Child process: the diagnostic library is
    loaded through MH_LIB, never beside the default one."""
    import os
    import subprocess
    import sys

    import metalhuffman_amd.build as B
    lib = B.diag_lib_path("spin0")
    assert os.path.exists(lib), "build() makes the diagnostic libraries"
    code = (
        "import sys, torch; sys.path.insert(0, %r)\n"
        "import metalhuffman_amd as mh\n"
        "from metalhuffman_amd import frames as F\n"
        "from metalhuffman_amd.encoder import Encoder\n"
        "assert mh.lib().mh_build_stamp().decode().startswith('diag:spin0:')\n"
        "img = torch.from_numpy(F.bigbridge()).cuda()\n"
        "enc = Encoder(img.shape[1], img.shape[0], 'cuda')\n"
        "bad = 0\n"
        "for _ in range(4):\n"
        "    try:\n"
        "        enc.encode(img)\n"
        "    except mh.MHError as e:\n"
        "        assert e.status == -7, e\n"
        "        bad += 1\n"
        "print('timeouts', bad)\n"
        "assert bad == 4\n" % B.ROOT)
    env = dict(os.environ, MH_LIB=lib, MH_ENCODE_KERNELS=path)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.parametrize("path", ["4", "1"])
def test_encoder_alternative_paths(mh, path):
    """The two-launch path is the default for frames of <= 512 code tiles; the
    four-kernel path (MH_ENCODE_KERNELS=4) stays selectable and byte-identical to the
    host codec; any other value (the removed one-launch path's "1" included) keeps the
    default. The knob is read once per process, so each path runs in a child process."""
    import os
    import subprocess
    import sys

    import metalhuffman_amd.build as B
    code = (
        "import sys, numpy as np, torch; sys.path.insert(0, %r)\n"
        "import metalhuffman_amd as mh\n"
        "from metalhuffman_amd import frames as F\n"
        "from metalhuffman_amd.encoder import Encoder\n"
        "bb = F.bigbridge()\n"
        "for img, init in ((bb, False), (np.ascontiguousarray(bb[:777, :1001]), True), (F.uniform_random(256, 320, 77), False)):\n"
        "    ref = mh.encode_frame(img, init_zero_delta=init)\n"
        "    enc = Encoder(img.shape[1], img.shape[0], 'cuda:0')\n"
        "    for _ in range(2):\n"
        "        a = enc.encode_async(torch.from_numpy(np.ascontiguousarray(img)).to('cuda:0'), 0, init)\n"
        "        r = a.result()\n"
        "        assert np.array_equal(r.canon, ref.canon)\n"
        "        assert np.array_equal(r.codes.cpu().numpy(), ref.codes)\n"
        "        assert np.array_equal(r.block_offsets.cpu().numpy().view(np.uint32), ref.block_offsets)\n"
        "        if init: assert np.array_equal(a.block_init.cpu().numpy(), ref.block_init)\n"
        "print('ok')\n" % B.ROOT)
    env = dict(os.environ, MH_ENCODE_KERNELS=path)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("path", ["2", "4"])
def test_async_encode_unzeroed_workspace_twice(mh, path):
    """without MH_ENCODE_WORKSPACE_ZEROED every call zeroes its per-call
    state. Two flags=0 calls on one workspace with DIFFERENT images must each give the
    host codec's bytes: the second call's packers must not take the first call's code
    table (whose words carried the same call tag before the table was zeroed too).
    Child process per path (MH_ENCODE_KERNELS is read once)."""
    import os
    import subprocess
    import sys

    import metalhuffman_amd.build as B
    code = (
        "import sys, ctypes, numpy as np, torch; sys.path.insert(0, %r)\n"
        "import metalhuffman_amd as mh\n"
        "from metalhuffman_amd import _native as N, frames as F\n"
        "from metalhuffman_amd.encoder import Encoder\n"
        "bb = F.bigbridge()\n"
        "imgs = [bb, F.uniform_random(1536, 2048, 9), np.ascontiguousarray(F.block_shuffle(bb, 3)), bb]\n"
        "enc = Encoder(2048, 1536, 'cuda:0')\n"
        "codes = torch.empty(enc.cap, dtype=torch.uint8, device='cuda:0')\n"
        "offs = torch.empty(enc.nb, dtype=torch.int32, device='cuda:0')\n"
        "canon = torch.empty(256, dtype=torch.uint8, device='cuda:0')\n"
        "meta = torch.zeros(2, dtype=torch.int64, device='cuda:0')\n"
        "base = enc.workspace.data_ptr(); al = (base + 255) // 256 * 256\n"
        "for k, img in enumerate(imgs):\n"
        "    ref = mh.encode_frame(img)\n"
        "    d = torch.from_numpy(np.ascontiguousarray(img)).to('cuda:0')\n"
        "    N.check(N.lib().mh_encode_frame_device_async(d.data_ptr(), 2048, 1536, 0, canon.data_ptr(),\n"
        "        codes.data_ptr(), codes.numel(), meta.data_ptr(), offs.data_ptr(), None, meta.data_ptr() + 8, al,\n"
        "        enc.workspace.numel() - (al - base), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), 'enc')\n"
        "    torch.cuda.synchronize()\n"
        "    n = int(meta[0].item())\n"
        "    assert int(meta[1].item()) == 0, (k, int(meta[1].item()))\n"
        "    assert np.array_equal(canon.cpu().numpy(), ref.canon), k\n"
        "    assert n == ref.codes.size, (k, n, ref.codes.size)\n"
        "    assert np.array_equal(codes[:n].cpu().numpy(), ref.codes), (k, int((codes[:n].cpu().numpy() != ref.codes).sum()))\n"
        "    assert np.array_equal(offs.cpu().numpy().view(np.uint32), ref.block_offsets), k\n"
        "print('ok')\n" % B.ROOT)
    env = dict(os.environ, MH_ENCODE_KERNELS=path)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr
