"""Config 5 over several GPUs of one node from ONE host process: frames streamed
from pinned host memory, round-robined over the devices by a native stream group
(mh_stream_group_*). Prints one JSON line: aggregate frames/s, decoded MB/s incl.
PCIe, and per-frame latencies. Every device's last frame is checked bit-exact.

    python scripts/stream_group_bench.py --devices 0,1,2,3,4,5,6,7 [--frames 4096]
    python scripts/stream_group_bench.py --devices 0,0        # one GPU, two members
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import metalhuffman_amd as mh  # noqa: E402
from metalhuffman_amd import decoder as D, frames as F  # noqa: E402
from metalhuffman_amd.stream import FrameStreamGroup, pinned_frame  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--devices", default="0")
    ap.add_argument("--frames", type=int, default=4096)
    ap.add_argument("--slots", type=int, default=2)
    ap.add_argument("--distinct", type=int, default=16)
    args = ap.parse_args()
    devices = [int(d) for d in args.devices.split(",")]
    bb = F.bigbridge()
    imgs = [F.block_shuffle(bb, 700 + i) for i in range(args.distinct)]
    efs = [mh.encode_frame(im) for im in imgs]
    t1, t2 = efs[0].tables()
    tabs = [D.DeviceTables.upload(t1, t2, torch.device("cuda", d)) for d in devices]
    hosts = [pinned_frame(ef) for ef in efs]
    g = FrameStreamGroup(tabs, 2048, 1536, max(ef.codes.size for ef in efs), slots=args.slots)
    for k in range(256):  # warm every member
        g.submit(*hosts[k % len(hosts)])
    g.synchronize()
    t0 = time.perf_counter()
    last = {}
    for k in range(args.frames):
        m, sl = g.submit(*hosts[k % len(hosts)])
        last[m] = (k % len(hosts), sl)
    g.synchronize()
    wall = time.perf_counter() - t0
    ok = all(torch.equal(g.output(m, sl)[:, :2048].cpu(), torch.from_numpy(imgs[i])) for m, (i, sl) in last.items())
    lat = []
    for k in range(500):
        t = time.perf_counter()
        m, sl = g.submit(*hosts[k % len(hosts)])
        g.wait(m, sl)
        lat.append((time.perf_counter() - t) * 1e6)
    g.close()
    print(json.dumps({"devices": devices, "frames": args.frames, "fps": round(args.frames / wall, 1),
                      "MBps_incl_pcie": round(args.frames * bb.size / wall / 1e6, 1),
                      "latency_us_p50": round(float(np.percentile(lat, 50)), 1),
                      "latency_us_p99": round(float(np.percentile(lat, 99)), 1),
                      "latency_us_max": round(max(lat), 1), "last_frames_bit_exact": ok}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
