"""Native stream (mh_stream_*) sustained rate vs slot count, beside bare pinned H2D copies of
the same size (back to back, and with an event record + cross-stream wait per copy)."""
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
nbytes = int(np.mean([ef.codes.size + 4 * ef.n_blocks for ef in efs]))
for slots in (2, 4):
    fs = FrameStream(tabs, 2048, 1536, max(ef.codes.size for ef in efs), slots=slots, device=dev)
    for rnd in range(3):
        n = 1024
        t0 = time.perf_counter()
        for i in range(n):
            c, o = hosts[i % 8]
            fs.submit(c, o)
        fs.synchronize()
        wall = time.perf_counter() - t0
    print(f"slots={slots}: {n / wall:8.1f} fps  {n * nbytes / wall / 1e9:6.2f} GB/s H2D", flush=True)
    fs.close()
# bare copies of one frame's bytes
src = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
s1 = torch.cuda.Stream(dev)
s2 = torch.cuda.Stream(dev)
for mode in ("bare", "event"):
    for rnd in range(3):
        n = 1024
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        with torch.cuda.stream(s1):
            for i in range(n):
                dst.copy_(src, non_blocking=True)
                if mode == "event":
                    e = torch.cuda.Event()
                    e.record(s1)
                    s2.wait_event(e)
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
    print(f"{mode} copies: {n / wall:8.1f} per s  {n * nbytes / wall / 1e9:6.2f} GB/s", flush=True)
