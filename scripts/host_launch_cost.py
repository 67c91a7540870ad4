"""Host cost of one decode launch through the Python wrapper (decoder.decode) and the
bare C-ABI call (mh_decode via ctypes, struct prepared once), vs the GPU time of the
same launches: are plain eager regions of the 64-frame batch host-bound?

    python scripts/host_launch_cost.py [n_frames_per_launch=64] [launches=256]"""
import ctypes
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import metalhuffman_amd as mh  # noqa: E402
from metalhuffman_amd import _native as N  # noqa: E402
from metalhuffman_amd import decoder as D  # noqa: E402
from metalhuffman_amd import frames as F  # noqa: E402

nf = int(sys.argv[1]) if len(sys.argv) > 1 else 64
K = int(sys.argv[2]) if len(sys.argv) > 2 else 256
dev = torch.device("cuda:0")
bb = F.bigbridge()
efs = [mh.encode_frame(F.block_shuffle(bb, s)) for s in range(nf)]
t1, t2 = efs[0].tables()
tabs = D.DeviceTables.upload(t1, t2, dev)
fr = D.DeviceFrames.pack(efs, dev)
out = torch.empty((nf, 1536, 2048), dtype=torch.uint8, device=dev)
for _ in range(16):
    D.decode(fr, tabs, out)
torch.cuda.synchronize()
for rep in range(2):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    for _ in range(K):
        D.decode(fr, tabs, out)
    th = time.perf_counter() - t0
    e1.record()
    torch.cuda.synchronize()
    tw = time.perf_counter() - t0
    print(f"decoder.decode x{K}: host {th / K * 1e6:.1f} us/launch, wall {tw / K * 1e6:.1f}, "
          f"GPU region {e0.elapsed_time(e1) / K * 1e3:.1f} us/launch")
# bare C-ABI call, struct built once
s = D._frame_struct(fr, tabs)
L = N.lib()
sp = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
optr, pitch = out.data_ptr(), 2048
for rep in range(2):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    for _ in range(K):
        L.mh_decode(ctypes.byref(s), optr, pitch, 1536 * pitch, sp)
    th = time.perf_counter() - t0
    e1.record()
    torch.cuda.synchronize()
    tw = time.perf_counter() - t0
    print(f"mh_decode x{K}: host {th / K * 1e6:.1f} us/launch, wall {tw / K * 1e6:.1f}, "
          f"GPU region {e0.elapsed_time(e1) / K * 1e3:.1f} us/launch")
# hipGraph replays (torch.cuda.CUDAGraph over decoder.decode): host cost of one replay of a
# graph of G launches, and whether back-to-back replays keep the GPU busy
for G in (1, 4, 16, 64, 256):
    if G > K:
        break
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(G):
            D.decode(fr, tabs, out)
    g.replay()
    torch.cuda.synchronize()
    R = max(1, K // G)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    for _ in range(R):
        g.replay()
    th = time.perf_counter() - t0
    e1.record()
    torch.cuda.synchronize()
    tw = time.perf_counter() - t0
    print(f"graph of {G} x{R} replays: host {th / (R * G) * 1e6:.1f} us/launch ({th / R * 1e6:.1f} per replay), "
          f"wall {tw / (R * G) * 1e6:.1f}, GPU region {e0.elapsed_time(e1) / (R * G) * 1e3:.1f} us/launch")
    del g
