"""Where the fixed cost of a short timed region goes (diagnostic, one GPU).

bench.py's headline wall clock at the driver's --steps 20 is K x kernel + a fixed
host cost (graph launch + synchronize). This probe times, for the single-frame
decode graph (K launches captured once):
  * wall of replay + synchronize, median of many, for K in (1, 20, 200);
  * the GPU region (HIP events) of the same replay;
  * an empty graph (one trivial kernel) for the pure host floor;
under the HIP device flag given on the command line (set before the context
exists): auto (default), spin, yield, blocking.

    python scripts/launch_overhead.py [auto|spin|yield|blocking]
"""
import ctypes
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FLAGS = {"auto": 0, "spin": 1, "yield": 2, "blocking": 4}
mode = sys.argv[1] if len(sys.argv) > 1 else "auto"
if FLAGS[mode]:
    hip = ctypes.CDLL("libamdhip64.so")
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(FLAGS[mode]))
    print(f"hipSetDeviceFlags({mode}) rc={rc}")

import numpy as np  # noqa: E402
import torch  # noqa: E402

import metalhuffman_amd as mh  # noqa: E402
from metalhuffman_amd import decoder as D  # noqa: E402
from metalhuffman_amd import frames as F  # noqa: E402

dev = torch.device("cuda", 0)
bb = F.bigbridge()
efs = [mh.encode_frame(F.block_shuffle(bb, s)) for s in range(8)]
t1, t2 = efs[0].tables()
tabs = D.DeviceTables.upload(t1, t2, dev)
launches = [D.DeviceFrames.pack([ef], dev) for ef in efs]
outs = [torch.empty((1, 1536, 2048), dtype=torch.uint8, device=dev) for _ in launches]
x = torch.zeros(1, device=dev)


def graph_of(k, fn):
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(k):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    return g


def dec(i):
    D.decode(launches[i % 8], tabs, outs[i % 8])


def tiny(i):
    x.add_(1)


def measure(g, n=200, sync="device"):
    walls, regions = [], []
    ev = torch.cuda.Event()
    for _ in range(n):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        g.replay()
        e1.record()
        if sync == "device":
            torch.cuda.synchronize()
        elif sync == "event":
            e1.synchronize()
        else:  # poll the event (busy wait in Python)
            while not e1.query():
                pass
        walls.append((time.perf_counter() - t0) * 1e6)
        regions.append(e0.elapsed_time(e1) * 1e3)
    return statistics.median(walls), statistics.median(regions), min(walls)


print(f"mode={mode}")
for k in (1, 20, 200):
    g = graph_of(k, dec)
    for sync in ("device", "event", "poll"):
        w, r, wmin = measure(g, n=100 if k == 200 else 300, sync=sync)
        print(f"decode graph K={k:3d} sync={sync:6s}: wall median {w:8.1f} us (min {wmin:8.1f}), "
              f"region {r:8.1f} us, wall-region {w - r:6.1f} us, per step {w / k:6.2f} us")
g = graph_of(1, tiny)
for sync in ("device", "event", "poll"):
    w, r, wmin = measure(g, sync=sync)
    print(f"tiny graph K=1 sync={sync:6s}: wall median {w:8.1f} us (min {wmin:8.1f}), region {r:6.1f} us")
