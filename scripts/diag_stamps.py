"""Phase timeline of one decode launch from a MH_DIAG_STAMPS=1 build (GPU, diagnostic).

    MH_LIB=ab/lib_diag.so python scripts/diag_stamps.py [--batch N]

Stamps (s_memrealtime, 100 MHz) per wave: 0 entry, 1 first header resolved,
2 LUT ready, 3 first span staged, 4 first tile decoded (stores issued),
5 loop done, 6 stores drained.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import metalhuffman_amd as mh  # noqa: E402
from metalhuffman_amd import _native as N, decoder as D, frames as F  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=1)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--tag", default="")
ap.add_argument("--clock", action="store_true",
                help="MH_DIAG_CLOCK build: slot 5 holds the decode's core-clock cycles (s_memtime)")
ap.add_argument("--tile8192", action="store_true", help="config 3: one 8192x8192 BigBridge mirror tile")
ap.add_argument("--random8192", action="store_true",
                help="config 3 stress: one 8192x8192 uniform-random frame (flat 8-bit table: the flat8 loop; "
                     "stamps 2 and 3 = 1, stamp 4 = first tile's codes landed and stores issued)")
ap.add_argument("--cold", action="store_true",
                help="stamp a launch of a second, never-decoded frame set after a 1 GiB cache flush (bench.py's cold rule)")
args = ap.parse_args()

lib = N.lib()
if not hasattr(lib, "mh_diag_stamps"):
    sys.exit("not a MH_DIAG_STAMPS build (set MH_LIB)")
bb = F.bigbridge()
if args.random8192:
    efs = [mh.encode_frame(F.uniform_random(8192, 8192, 1234))]
    efs2 = [mh.encode_frame(F.block_shuffle(F.uniform_random(8192, 8192, 1234), 100))] if args.cold else efs
elif args.tile8192:
    base = F.mirror_tile(bb, 8192, 8192)
    efs = [mh.encode_frame(base)]
    efs2 = [mh.encode_frame(F.block_shuffle(base, 100))] if args.cold else efs
else:
    efs = [mh.encode_frame(F.block_shuffle(bb, i) if i else bb) for i in range(args.batch)]
    efs2 = ([mh.encode_frame(F.block_shuffle(bb, 1000 + i)) for i in range(args.batch)] if args.cold else efs)
t1, t2 = efs[0].tables()
tabs = D.DeviceTables.upload(t1, t2, "cuda")
fr = D.DeviceFrames.pack(efs, "cuda")
fr2 = D.DeviceFrames.pack(efs2, "cuda")
out = D.decode(fr, tabs)
out2 = torch.empty_like(out)
for _ in range(args.reps):
    D.decode(fr, tabs, out)
if args.cold:  # evict the Infinity Cache and L2s; the stamped launch decodes frames nothing touched yet
    fa = torch.empty(512 << 20, dtype=torch.uint8, device="cuda").fill_(1)
    torch.empty_like(fa).copy_(fa)
    del fa
torch.cuda.synchronize()
s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s0.record()
D.decode(fr2, tabs, out2)
s1.record()
torch.cuda.synchronize()
n = 8192 * 8
buf = (ctypes.c_ulonglong * n)()
assert lib.mh_diag_stamps(buf, ctypes.c_size_t(n)) == n
st = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 8)
live = st[:, 0] > 0
st = st[live]
t0 = st[:, 0].min()
print(f"launch event time {s0.elapsed_time(s1) * 1e3:.2f} us; waves {live.sum()}")
if args.clock:  # slot 5 = s_memtime cycles between stamps 3 and 4 (staged tiles only)
    cyc = st[:, 5].astype(np.int64)
    us = (st[:, 4].astype(np.int64) - st[:, 3].astype(np.int64)) * 0.01
    ok = (cyc > 0) & (us > 0)
    mhz = cyc[ok] / us[ok]
    print(f"decode core cycles p50 {np.median(cyc[ok]):.0f} p90 {np.percentile(cyc[ok], 90):.0f}; "
          f"per symbol p50 {np.median(cyc[ok]) / 64:.1f}; clock MHz p10 {np.percentile(mhz, 10):.0f} "
          f"p50 {np.median(mhz):.0f} p90 {np.percentile(mhz, 90):.0f}")
    st[:, 5] = st[:, 4]
names = ["entry", "hdr", "lut", "staged", "tile0", "loop", "drain"]
for i, nm in enumerate(names):
    v = (st[:, i].astype(np.int64) - int(t0)) * 0.01
    print(f"{nm:7s} us  min {v.min():7.2f}  p50 {np.median(v):7.2f}  p90 {np.percentile(v, 90):7.2f}  max {v.max():7.2f}")
loop_end = (st[:, 5].astype(np.int64) - int(t0)) * 0.01
print("loop end per wave: p10 %.2f p50 %.2f p90 %.2f p99 %.2f max %.2f us" % tuple(np.percentile(loop_end, [10, 50, 90, 99, 100])))
for a, b in [(0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (5, 6)]:
    d = (st[:, b].astype(np.int64) - st[:, a].astype(np.int64)) * 0.01
    print(f"{names[a]}->{names[b]:7s} p50 {np.median(d):7.2f}  p90 {np.percentile(d, 90):7.2f}  max {d.max():7.2f}")
# start / steady / drain: until the median wave has its first span staged; from then
# until the first 10 % of waves have finished their last tile; from then to the last drain
T = lambda i: (st[:, i].astype(np.int64) - int(t0)) * 0.01
start, fin10, end = float(np.median(T(3))), float(np.percentile(T(5), 10)), float(T(6).max())
print(f"decomposition: start {start:.2f} us, steady {fin10 - start:.2f} us, drain {end - fin10:.2f} us "
      f"(end {end:.2f} us)")
out_npz = os.path.join(ROOT, "gpurun_out", f"stamps_b{args.batch}{args.tag}{'_cold' if args.cold else ''}.npz")
os.makedirs(os.path.dirname(out_npz), exist_ok=True)
np.savez(out_npz, stamps=np.frombuffer(buf, dtype=np.uint64).reshape(-1, 8))
