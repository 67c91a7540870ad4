"""Batched device encoder (mh_encode_frames_device_async) on n BigBridge block
shuffles per call: wall and HIP-event time per frame, calls back to back on one
stream; run under rocprofv3 --kernel-trace --stats for the per-kernel split
(enc_split_kernel / enc_tree_batch_kernel / enc_pack_wave_kernel).

    python scripts/enc_batch_profile.py [n_frames] [calls]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import metalhuffman_amd as mh  # noqa: E402
from metalhuffman_amd import frames as F  # noqa: E402
from metalhuffman_amd.encoder import BatchEncoder  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 8
bb = F.bigbridge()
dev = torch.device("cuda:0")
imgs = np.stack([F.block_shuffle(bb, 700 + k) for k in range(n)])
g = torch.from_numpy(imgs).to(dev)
enc = BatchEncoder(bb.shape[1], bb.shape[0], n, dev)
a = enc.encode_async(g)
torch.cuda.synchronize()
ref = mh.encode_frame(imgs[n - 1])
if not os.environ.get("MH_PROFILE_NO_CHECK"):  # diagnostic variants (wrong output on purpose) skip it
    assert int((a.status != 0).sum().item()) == 0
    for f in (0, n - 1):
        assert np.array_equal(a.frame(f).codes.cpu().numpy(), mh.encode_frame(imgs[f]).codes), f
alg = bb.size + ref.codes.size + 4 * ref.n_blocks  # pixels in, codes + offsets out
print(f"alg_bytes {alg * n} per call of {n} frames")
for rep in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(calls):
        enc.encode_async(g)
    e1.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / (calls * n)
    ev = e0.elapsed_time(e1) * 1e-3 / (calls * n)
    print(f"batch {n}: {ev * 1e6:.2f} us/frame (events), {wall * 1e6:.2f} us/frame (wall), "
          f"{alg / ev / 1e9:.1f} GB/s algorithmic ({alg / ev / 8e12:.4f} of 8 TB/s)")
