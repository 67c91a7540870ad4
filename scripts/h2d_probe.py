"""Host-to-device bandwidth from pinned memory (config 5's shared resource): one frame's
bytes (codes + offsets, ~2.12 MB) copied back to back on one stream, split over 2 / 4
streams (each copy a 1/k slice, all slices of a frame in flight together), and 64 MB copies
(the link's large-transfer rate). Decides whether mh_stream should spread a frame's H2D
over several copy streams (several SDMA engines).

    python scripts/h2d_probe.py
"""
import time

import torch

dev = torch.device("cuda", 0)
nbytes = 2_120_000
src = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
streams = [torch.cuda.Stream(dev) for _ in range(8)]


def run(k, n=1024, size=nbytes, s_src=src, s_dst=dst):
    sl = [(i * size // k, (i + 1) * size // k) for i in range(k)]
    best = 0.0
    for rnd in range(3):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for it in range(n):
            for j, (a, b) in enumerate(sl):
                with torch.cuda.stream(streams[j]):
                    s_dst[a:b].copy_(s_src[a:b], non_blocking=True)
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        best = max(best, n * size / wall / 1e9)
    return best


for k in (1, 2, 4, 8):
    print(f"frame-size copies ({nbytes} B) split over {k} stream(s): {run(k):6.2f} GB/s", flush=True)
big = 64 << 20
bs = torch.empty(big, dtype=torch.uint8).pin_memory()
bd = torch.empty(big, dtype=torch.uint8, device=dev)
for k in (1, 2, 4):
    print(f"64 MB copies split over {k} stream(s): {run(k, n=32, size=big, s_src=bs, s_dst=bd):6.2f} GB/s", flush=True)
