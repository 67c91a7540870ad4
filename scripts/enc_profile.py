"""Run the device-only encoder on BigBridge-shuffled frames (for rocprofv3
--kernel-trace --stats: per-kernel times of split / tree / zero / blen / scan / pack)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from metalhuffman_amd import frames as F  # noqa: E402
from metalhuffman_amd.encoder import Encoder  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 64
bb = F.bigbridge()
dev = torch.device("cuda:0")
imgs = [torch.from_numpy(F.block_shuffle(bb, 900 + k)).to(dev) for k in range(4)]
enc = Encoder(bb.shape[1], bb.shape[0], dev)
codes = [torch.empty(enc.cap, dtype=torch.uint8, device=dev) for _ in range(4)]
for k in range(8):
    enc.encode_async(imgs[k % 4], codes=codes[k % 4])
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(reps):
    enc.encode_async(imgs[k % 4], codes=codes[k % 4])
torch.cuda.synchronize()
print(f"async encode {1e6 * (time.perf_counter() - t0) / reps:.1f} us/frame")

# the same encodes enqueued behind bench.py's launch gate before the clock starts:
# device time per frame without the host's enqueue cost (Python + 4 launches)
from bench import GATE  # noqa: E402
if GATE.ok():
    for rep in range(2):
        torch.cuda.synchronize()
        GATE.arm(torch.cuda.current_stream().cuda_stream)
        te = time.perf_counter()
        for k in range(reps):
            enc.encode_async(imgs[k % 4], codes=codes[k % 4])
        t0 = time.perf_counter()
        print(f"host enqueue {1e6 * (t0 - te) / reps:.1f} us/frame")
        GATE.open()
        torch.cuda.synchronize()
        print(f"gated async encode {1e6 * (time.perf_counter() - t0) / reps:.1f} us/frame")

# the same encodes captured once in a hipGraph and replayed (launch path of a
# GPU-resident producer that re-encodes frames of one size)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for k in range(64):
        enc.encode_async(imgs[k % 4], codes=codes[k % 4])
g.replay()
torch.cuda.synchronize()
for rep in range(2):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"graph replay encode {e0.elapsed_time(e1) * 1e3 / 64:.1f} us/frame")

if len(sys.argv) > 2 and sys.argv[2] == "stamps":
    # library built with -DMH_TREE_STAMPS=1: s_memtime at the tree kernel's phase
    # boundaries in meta[2..10] (either path: the tree runs in enc_tree_kernel or workgroup 0)
    from metalhuffman_amd import _native as N
    # meta's offset in the workspace: mh_encode.hip carve() (sym, blen, tsum, hist, table, meta)
    a256 = lambda x: (x + 255) // 256 * 256
    nb = ((bb.shape[1] + 7) // 8) * ((bb.shape[0] + 7) // 8)
    moff = a256(nb * 64) + a256(nb * 4) + a256((nb + 255) // 256 * 4) + a256(8 * 256 * 8) + a256(256 * 4)
    base = enc.workspace.data_ptr()
    off = (base + 255) // 256 * 256 - base + moff
    for k in range(3):
        enc.encode_async(imgs[k], codes=codes[k])
        torch.cuda.synchronize()
        m = enc.workspace[off: off + 88].cpu().view(torch.int64).tolist()
        st = m[2:11]
        print("tree phases (s_memtime clocks): load", st[1] - st[0], "rank", st[2] - st[1], "merge", st[3] - st[2],
              "jump-init", st[4] - st[3], "jump+lengths", st[5] - st[4], "ballots", st[6] - st[5],
              "first-codes", st[7] - st[6], "table", st[8] - st[7], "total", st[8] - st[0])
