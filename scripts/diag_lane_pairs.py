"""Where the lane-pair kernel's bytes differ from the input (GPU diagnostic): per
mismatched block, the differing byte positions, the emulator's split (ia, jb) and
whether the difference is a constant (delta rebase) or a shift (split indices)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import metalhuffman_amd as mh  # noqa: E402
from metalhuffman_amd import decoder as D, frames as F  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import emu_lane_pairs as E  # noqa: E402

bb = F.bigbridge()
ef = mh.encode_frame(bb)
t1, t2 = ef.tables()
tabs = D.DeviceTables.upload(t1, t2, "cuda:0")
fr = D.DeviceFrames.pack([ef], "cuda:0")
out = D.decode(fr, tabs, extra_flags=mh.MH_FLAG_LANE_PAIRS)
torch.cuda.synchronize()
img = out[0, :, : fr.width].cpu().numpy()
bw, bh = 256, 192
got = img.reshape(bh, 8, bw, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
ref = bb.reshape(bh, 8, bw, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
bad = np.nonzero((got != ref).any(1))[0]
print("mismatched blocks", bad.size, "of", ref.shape[0])
if bad.size:
    print("first", bad[:20].tolist())
    lanes = np.bincount(bad % 32, minlength=32)
    print("by block index mod 32", lanes.tolist())
    for b in bad[:8]:
        d = np.nonzero(got[b] != ref[b])[0]
        diff = ((got[b].astype(int) - ref[b].astype(int)) % 256)[d]
        print(f"block {b}: bytes {d.min()}..{d.max()} ({d.size}), diffs {np.unique(diff)[:8].tolist()}")
        print("   got", got[b][:16].tolist(), "ref", ref[b][:16].tolist())
