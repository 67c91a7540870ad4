"""Kernel time of one-frame decode launches WITHOUT output checks (GPU, diagnostic).

    MH_LIB=ab/lib_<variant>.so python scripts/time_frame.py [--frames 16] [--k 200] [--reps 3]

For diagnostic builds whose output is wrong on purpose (e.g. -DMH_DIAG_BROADCAST_LUT=1:
every lane reads table entry 0, so the lookups are conflict-free broadcasts and the step
chain keeps its shape), which bench.py refuses to time. K launches over distinct
block-shuffled BigBridge frames, captured in one hipGraph and replayed between an event
pair (a Python launch loop would be host-bound: ~8 us per call against ~5.5 us kernels).
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import metalhuffman_amd as mh  # noqa: E402
from metalhuffman_amd import _native as N, decoder as D, frames as F  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=16)
ap.add_argument("--k", type=int, default=200)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--batch", type=int, default=1, help="frames per launch (64: the config-4 shard)")
ap.add_argument("--tag", default=os.path.basename(os.environ.get("MH_LIB", "default")))
ap.add_argument("--random", action="store_true",
                help="uniform-random 2048x1536 frames (a flat 8-bit table) instead of BigBridge shuffles")
args = ap.parse_args()

N.lib()
bb = F.bigbridge()
if args.random:
    efs = [mh.encode_frame(F.uniform_random(1536, 2048, 4000 + i)) for i in range(args.frames)]
else:
    efs = [mh.encode_frame(F.block_shuffle(bb, i) if i else bb) for i in range(args.frames)]
t1, t2 = efs[0].tables()
tabs = D.DeviceTables.upload(t1, t2, "cuda")
if args.batch > 1:
    frs = [D.DeviceFrames.pack([efs[(j + i) % len(efs)] for i in range(args.batch)], "cuda") for j in range(2)]
else:
    frs = [D.DeviceFrames.pack([e], "cuda") for e in efs]
outs = [D.decode(f, tabs) for f in frs]
for i in range(64):
    D.decode(frs[i % len(frs)], tabs, outs[i % len(frs)])
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
side = torch.cuda.Stream()
with torch.cuda.stream(side):
    with torch.cuda.graph(g, stream=side):
        for i in range(args.k):
            D.decode(frs[i % len(frs)], tabs, outs[i % len(frs)])
torch.cuda.synchronize()
g.replay()
torch.cuda.synchronize()
best = None
for _ in range(args.reps):
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0.record()
    g.replay()
    s1.record()
    torch.cuda.synchronize()
    us = s0.elapsed_time(s1) * 1e3 / args.k
    best = us if best is None else min(best, us)
    print(f"{args.tag}: {us:.3f} us per launch ({args.k} launches)", flush=True)
print(f"{args.tag}: best {best:.3f} us per launch")
