"""Host-side cost of the native stream's submit (copy + decode graph + two timing events per
frame) vs the device-side rate: per-call wall of mh_stream_submit at 4 slots, and the
sustained rate. If the host's per-call time approaches the frame period, submission -- not
PCIe -- is config 5's limit.

    python scripts/h2d_probe3.py
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import metalhuffman_amd as mh  # noqa: E402
from metalhuffman_amd import decoder as D, frames as F  # noqa: E402
from metalhuffman_amd.stream import FrameStream, pinned_frame  # noqa: E402

dev = torch.device("cuda", 0)
bb = F.bigbridge()
efs = [mh.encode_frame(F.block_shuffle(bb, s)) for s in range(8)]
t1, t2 = efs[0].tables()
tabs = D.DeviceTables.upload(t1, t2, dev)
hosts = [pinned_frame(ef) for ef in efs]
fb = int(np.mean([ef.codes.size + 4 * ef.n_blocks for ef in efs]))
fs = FrameStream(tabs, 2048, 1536, max(ef.codes.size for ef in efs), slots=4, device=dev)
for rnd in range(3):
    n = 2048
    per = np.empty(n)
    t0 = time.perf_counter()
    for i in range(n):
        c, o = hosts[i % 8]
        a = time.perf_counter()
        fs.submit(c, o)
        per[i] = time.perf_counter() - a
    t_enq = time.perf_counter() - t0
    fs.synchronize()
    wall = time.perf_counter() - t0
    print(f"slots=4: {n / wall:8.0f} fps sustained ({n * fb / wall / 1e9:.1f} GB/s); submit call p50 "
          f"{np.median(per) * 1e6:.1f} us p90 {np.percentile(per, 90) * 1e6:.1f} us mean {per.mean() * 1e6:.1f} us; "
          f"enqueue of all {t_enq * 1e3:.1f} ms of {wall * 1e3:.1f} ms", flush=True)
fs.close()
