"""Phase stamps of the fused encoder kernel (library built with -DMH_CODE_STAMPS=1,
loaded with MH_LIB): per packing workgroup the time it started, saw the table flag,
had the table, finished -- relative to workgroup 0's start (s_memrealtime, 100 MHz)."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from metalhuffman_amd import _native as N  # noqa: E402
from metalhuffman_amd import frames as F  # noqa: E402
from metalhuffman_amd.encoder import Encoder  # noqa: E402

bb = F.bigbridge()
dev = torch.device("cuda:0")
img = torch.from_numpy(F.block_shuffle(bb, 901)).to(dev)
enc = Encoder(bb.shape[1], bb.shape[0], dev)
lib = N.lib()
lib.mh_diag_code_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
lib.mh_diag_split_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
nwg = 1 + (enc.nb + 127) // 128
imgs = [torch.from_numpy(F.block_shuffle(bb, 900 + k)).to(dev) for k in range(4)]
codes = [torch.empty(enc.cap, dtype=torch.uint8, device=dev) for _ in range(4)]
for rep in range(6):
    torch.cuda.synchronize()
    lib.mh_diag_code_stamps_reset()
    if rep < 3:  # one frame alone
        enc.encode_async(img)
    else:        # the last of 64 frames enqueued back to back
        for k in range(64):
            enc.encode_async(imgs[k % 4], codes=codes[k % 4])
    torch.cuda.synchronize()
    st = np.zeros(1024 * 8, np.uint64)
    lib.mh_diag_code_stamps(st.ctypes.data, st.size)
    ss = np.zeros(1024 * 8, np.uint64)
    lib.mh_diag_split_stamps(ss.ctypes.data, ss.size)
    ss = ss.reshape(1024, 8)[: nwg - 1, :5].astype(np.int64)
    st = st.reshape(1024, 8)[:nwg].astype(np.int64)
    ids = st[1:, 7].copy()
    st[:, 7] = 0
    t0 = st[0, 0]
    us = (st - t0) / 100.0
    p = us[1:]
    q = lambda a: f"{np.min(a):6.2f} {np.median(a):6.2f} {np.max(a):6.2f}"
    s0 = ss[:, 0].min()
    sq = lambda a: f"{np.min(a):6.2f} {np.median(a):6.2f} {np.max(a):6.2f}"
    ssu = (ss - s0) / 100.0
    print(f"rep {rep}: split (us from its first workgroup) start {sq(ssu[:,0])} loaded {sq(ssu[:,1])}"
          f" counted {sq(ssu[:,2])} reduced {sq(ssu[:,3])} end {sq(ssu[:,4])}; code wg0 start at {(t0 - s0) / 100:.2f}")
    print(f"rep {rep}: wg0 tree done {us[0,1]:.2f} flag-store {us[0,2]:.2f} end {us[0,3]:.2f} us")
    print(f"   pack start  min/med/max {q(p[:,0])}")
    print(f"   flag seen   {q(p[:,1])}")
    print(f"   table in    {q(p[:,2])}")
    print(f"   scanned     {q(p[:,4])}")
    print(f"   packed(LDS) {q(p[:,5])}")
    print(f"   stores out  {q(p[:,6])}")
    print(f"   end         {q(p[:,3])}")
    late = p[:, 0] > 5.0
    cu = (ids >> 32) * 100000 + (ids & 0xFFFFFFFF)
    print(f"   late starters {int(late.sum())} of {len(late)}; distinct CUs {len(set(cu.tolist()))};"
          f" max WGs on one CU {max(np.unique(cu, return_counts=True)[1])}; late on CUs already used:"
          f" {int(np.isin(cu[late], cu[~late]).sum())}")
