"""Native stream (mh_stream_*) throughput vs warm-up length and graph/direct launch."""
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import metalhuffman_amd as mh
from metalhuffman_amd import decoder as D, frames as F
from metalhuffman_amd.stream import FrameStream, pinned_frame

dev = torch.device("cuda", 0)
bb = F.bigbridge()
efs = [mh.encode_frame(F.block_shuffle(bb, s)) for s in range(8)]
t1, t2 = efs[0].tables()
tabs = D.DeviceTables.upload(t1, t2, dev)
hosts = [pinned_frame(ef) for ef in efs]
fs = FrameStream(tabs, 2048, 1536, max(ef.codes.size for ef in efs), slots=2, device=dev)
mode = os.environ.get("MH_STREAM_GRAPHS", "1")
for rnd in range(6):
    n = 256
    t0 = time.perf_counter()
    for i in range(n):
        c, o = hosts[i % 8]
        fs.submit(c, o)
    t_issue = time.perf_counter() - t0
    fs.synchronize()
    wall = time.perf_counter() - t0
    print(f"graphs={mode} round {rnd}: {n / wall:8.1f} fps  issue {t_issue / n * 1e6:6.1f} us/frame")
fs.close()
