"""Config-5 pipeline probe: throughput of bench.stream_h2d-style double buffering with
and without per-frame timing events and graphs (diagnostic)."""
import sys, os, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import metalhuffman_amd as mh
from metalhuffman_amd import decoder as D, frames as F

dev = torch.device("cuda", 0)
bb = F.bigbridge()
efs = [mh.encode_frame(F.block_shuffle(bb, s)) for s in range(8)]
t1, t2 = efs[0].tables()
tables = D.DeviceTables.upload(t1, t2, dev)
W, H = 2048, 1536
cap = max(int(np.ceil(ef.codes.size / 16)) * 16 for ef in efs)
nb = efs[0].n_blocks
hc = [torch.zeros(cap, dtype=torch.uint8).pin_memory() for _ in efs]
ho = [torch.from_numpy(ef.block_offsets.view(np.int32).copy()).pin_memory() for ef in efs]
for h, ef in zip(hc, efs):
    h[: ef.codes.size].copy_(torch.from_numpy(ef.codes))
slots = []
for _ in range(2):
    fr = D.DeviceFrames(W, H, 1, torch.zeros(nb, dtype=torch.int32, device=dev),
                        torch.zeros(cap, dtype=torch.uint8, device=dev), None)
    slots.append((fr, torch.empty((1, H, W), dtype=torch.uint8, device=dev)))
cs, ks = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
graphs = []
for fr, out in slots:
    with torch.cuda.stream(ks):
        D.decode(fr, tables, out, stream=ks)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=ks):
        D.decode(fr, tables, out, stream=ks)
    graphs.append(g)
torch.cuda.synchronize(dev)
free = [torch.cuda.Event() for _ in range(2)]
copied = [torch.cuda.Event() for _ in range(2)]


def run(n, use_graph, timing):
    tin = [torch.cuda.Event(enable_timing=True) for _ in range(n)] if timing else None
    tout = [torch.cuda.Event(enable_timing=True) for _ in range(n)] if timing else None
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(n):
        s, j = i % 2, i % len(efs)
        fr, out = slots[s]
        with torch.cuda.stream(cs):
            if i >= 2:
                cs.wait_event(free[s])
            if timing:
                tin[i].record(cs)
            fr.codes.copy_(hc[j], non_blocking=True)
            fr.block_offsets.copy_(ho[j], non_blocking=True)
            copied[s].record(cs)
        with torch.cuda.stream(ks):
            ks.wait_event(copied[s])
            if use_graph:
                graphs[s].replay()
            else:
                D.decode(fr, tables, out, stream=ks)
            free[s].record(ks)
            if timing:
                tout[i].record(ks)
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    lat = ""
    if timing:
        l = sorted(a.elapsed_time(b) * 1e3 for a, b in zip(tin, tout))
        lat = f" lat p50 {l[n//2]:.1f} us p99 {l[int(n*0.99)]:.1f}"
    print(f"graph={use_graph} timing={timing}: {n/wall:8.1f} fps, issue {t_issue/n*1e6:6.1f} us/frame{lat}")


for args in ((True, False), (False, False), (True, True), (False, True)):
    run(32, *args)
    run(512, *args)
