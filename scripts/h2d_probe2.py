"""H2D from pinned memory, whole frames (~2.12 MB each) round-robined over k streams (as
mh_stream's per-slot streams do), every rep printed; then the native stream's sustained
rate at 2 / 4 / 8 slots (copy + decode graph per frame).

    python scripts/h2d_probe2.py
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
dev = torch.device("cuda", 0)
nbytes = 2_120_000
srcs = [torch.empty(nbytes, dtype=torch.uint8).pin_memory() for _ in range(8)]
dsts = [torch.empty(nbytes, dtype=torch.uint8, device=dev) for _ in range(8)]
streams = [torch.cuda.Stream(dev) for _ in range(8)]
for k in (1, 2, 3, 4, 8):
    rates = []
    for rnd in range(5):
        n = 1024
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(n):
            j = i % k
            with torch.cuda.stream(streams[j]):
                dsts[j].copy_(srcs[i % 8], non_blocking=True)
        torch.cuda.synchronize(dev)
        rates.append(n * nbytes / (time.perf_counter() - t0) / 1e9)
    print(f"whole frames round-robin over {k} stream(s): " + " ".join(f"{r:5.1f}" for r in rates) + " GB/s",
          flush=True)

import metalhuffman_amd as mh  # noqa: E402
from metalhuffman_amd import decoder as D, frames as F  # noqa: E402
from metalhuffman_amd.stream import FrameStream, pinned_frame  # noqa: E402

bb = F.bigbridge()
efs = [mh.encode_frame(F.block_shuffle(bb, s)) for s in range(8)]
t1, t2 = efs[0].tables()
tabs = D.DeviceTables.upload(t1, t2, dev)
hosts = [pinned_frame(ef) for ef in efs]
fb = int(np.mean([ef.codes.size + 4 * ef.n_blocks for ef in efs]))
for slots in (2, 4, 8):
    fs = FrameStream(tabs, 2048, 1536, max(ef.codes.size for ef in efs), slots=slots, device=dev)
    rates = []
    for rnd in range(4):
        n = 1024
        t0 = time.perf_counter()
        for i in range(n):
            c, o = hosts[i % 8]
            fs.submit(c, o)
        fs.synchronize()
        rates.append(n / (time.perf_counter() - t0))
    fs.close()
    print(f"mh_stream slots={slots}: " + " ".join(f"{r:8.0f}" for r in rates) + f" fps ({max(rates) * fb / 1e9:.1f} GB/s best)",
          flush=True)
